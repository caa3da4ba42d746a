#!/bin/bash
# round 3, call 9: the plugin worker's lifecycle test alone (diagnostic words in the failure message)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c9; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -v --timeout 250 --timeout-method thread > "$O/worker.log" 2>&1
rc=$?; grep -E "PASS|FAIL|stopped|Error|error" "$O/worker.log" | head -20; exit $rc
