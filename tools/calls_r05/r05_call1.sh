#!/bin/bash
# round 5, call 1: the new parity tests (queue-slot reuse, configs[3] whole key runs + mutants, N>1 bench line with its
# CPU baseline), the default bench line (new copy-kernel bar, full-host extrapolation), then the guard-page test last
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c1; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_c4_keyruns.py tests/test_gpu_bench.py -x -v \
    --timeout 300 --timeout-method thread > "$O/new_tests.log" 2>&1
rc=$?; tail -3 "$O/new_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/new_tests.log" | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py > "$O/bench_c2.log" 2> "$O/bench_c2.err" || { tail "$O/bench_c2.err"; exit 1; }
tail -c 600 "$O/bench_c2.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 120 --timeout-method thread > "$O/guard.log" 2>&1
rc=$?; tail -3 "$O/guard.log"; exit $rc
