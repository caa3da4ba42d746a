#!/bin/bash
# round 3, call 3: split records with workgroup-scope fences (call 2: agent scope wrote back / invalidated the L2 per
# split record, c4 427 GiB/s); parity of the split / supp / dealing tests, the c4 threshold sweep, plugin phase stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c3; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_dealing.py "tests/test_gpu_parity.py" -k "split or dealing or supp or header" \
  -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for rep in 1 2; do
  for pct in 0 75 50 100 125; do
    echo "PTLS_HIP_SPLIT_PCT=$pct" >> "$O/split_c4.log"
    PTLS_HIP_SPLIT_PCT=$pct timeout -k 10 240 python tools/time_cfg.py hsig-picotls_amd/libptls_hip.so --config c4 --clock --reps 6 \
      >> "$O/split_c4.log" 2>&1 || { echo "split $pct rc=$?"; exit 1; }
  done
done
grep -v amdgpu.ids "$O/split_c4.log"
timeout -k 10 300 python tools/plugin_stamps.py > "$O/stamps.log" 2>&1 || { echo "stamps rc=$?"; tail -20 "$O/stamps.log"; exit 1; }
tail -1 "$O/stamps.log"
