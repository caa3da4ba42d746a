#!/bin/bash
# round 3, call 2: the GPU suite (split records, multi-device node, 2-rank bench, host-buffer safety + everything
# before), then the same-box c2 A/B (r01 / r02 / HEAD), the c4 split threshold sweep, one default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c2; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_node.py tests/test_gpu_bench.py -x -v --timeout 300 \
  --timeout-method thread > "$O/pytest_new.log" 2>&1 || { echo "pytest new rc=$?"; tail -40 "$O/pytest_new.log"; exit 1; }
tail -3 "$O/pytest_new.log"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
LIBS=(ab/r01/hsig-picotls_amd/libptls_hip.so ab/r02/hsig-picotls_amd/libptls_hip.so hsig-picotls_amd/libptls_hip.so)
for rep in 1 2; do
  for L in "${LIBS[@]}"; do
    timeout -k 10 180 python tools/time_cfg.py "$L" --config c2 --clock --reps 11 >> "$O/ab_c2.log" 2>&1 || { echo "time_cfg $L rc=$?"; exit 1; }
  done
done
cat "$O/ab_c2.log"
for rep in 1 2; do
  for pct in 0 75 50 100; do
    echo "PTLS_HIP_SPLIT_PCT=$pct" >> "$O/split_c4.log"
    PTLS_HIP_SPLIT_PCT=$pct timeout -k 10 240 python tools/time_cfg.py hsig-picotls_amd/libptls_hip.so --config c4 --clock --reps 6 \
      >> "$O/split_c4.log" 2>&1 || { echo "split $pct rc=$?"; exit 1; }
  done
done
cat "$O/split_c4.log"
timeout -k 10 600 python bench.py > "$O/bench_c2.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench_c2.log"; exit 1; }
tail -1 "$O/bench_c2.log"
