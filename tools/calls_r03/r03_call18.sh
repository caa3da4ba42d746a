#!/bin/bash
# round 3, call 18: planner at G = 32 for key runs of <= 64 records (configs[3]): GPU suite, bench c4 (full line)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c18; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 500 python bench.py --config c4 > "$O/bench_c4.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench_c4.log"; exit 1; }
tail -1 "$O/bench_c4.log" | cut -c1-1500
