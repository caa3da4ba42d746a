#!/bin/bash
# round 5, call 3: copy-shape probe (the roofline's achievable-HBM bar), the guard-page test, the ADVICE r04 fixes' tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c3; mkdir -p "$O"
timeout -k 10 240 tools/copy_probe/copy_probe > "$O/copy_probe.log" 2>&1 || { tail "$O/copy_probe.log"; exit 1; }
cat "$O/copy_probe.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 120 --timeout-method thread > "$O/guard.log" 2>&1
rc=$?; tail -25 "$O/guard.log"; [ $rc -eq 0 ] || exit $rc
# the ADVICE changes (engine memory pool, worker publication flag, stream-ordered key buffers, ECB launch path)
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_tls13.py tests/test_gpu_queue.py tests/test_gpu_node.py \
    -x -q --timeout 300 --timeout-method thread > "$O/advice_tests.log" 2>&1
rc=$?; tail -3 "$O/advice_tests.log"; exit $rc
