#!/bin/bash
# round 3, call 25: sparse-kernel threshold 20: GPU suite, smoke, c4 at 16 / 32 lanes on one box (alternating x2), bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c25; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
P=$R/hsig-picotls_amd/libptls_hip.so
for rep in 1 2; do
  for G in 16 32; do
    timeout -k 10 200 python tools/time_cfg.py $P --config c4 --lanes $G --reps 5 >> "$O/c4.log" 2>&1 || { echo "rc=$?"; exit 1; }
  done
done
grep -v amdgpu.ids "$O/c4.log"
timeout -k 10 400 python bench.py > "$O/bench.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench.log"; exit 1; }
grep '"metric"' "$O/bench.log" | cut -c1-500
