#!/bin/bash
# round 4, call 14 (second session, tree rebuilt in a fresh container): GPU suite, smoke, default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c14; mkdir -p "$O"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python -u bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" && tail -1 "$O/bench_c2.json" || { tail "$O/bench_c2.err"; exit 1; }
