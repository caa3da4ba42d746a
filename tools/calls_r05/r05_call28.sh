#!/bin/bash
# round 5, call 28: the planner's lanes-per-record choices pinned (tests/test_gpu_planner.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c28; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_planner.py -m gpu -v --timeout 120 --timeout-method thread > "$O/planner.log" 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed" "$O/planner.log" | tail -16; exit $rc
