#!/bin/bash
# round 4, call 7: the worker with constant-address-space (scalar) key loads, WITHOUT scratch and on
# the pooled-slot design, through the lifecycle / threads / size tests ONCE; then its per-call latency against the
# shipping worker (vector key loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c7; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so; W=$R/hsig-picotls_amd/variants/libptls_hip_wconst.so
PTLS_HIP_LIB=$W timeout -k 10 400 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_plugin_sizes.py -x -v --timeout 300 --timeout-method thread > "$O/wconst_tests.log" 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|error" "$O/wconst_tests.log" | tail -12; [ $rc -eq 0 ] || exit $rc
for L in $P $W $P $W; do
  PTLS_HIP_LIB=$L timeout -k 10 120 python -u tools/plugin_probe.py > "$O/probe.json" 2>/dev/null || exit 1
  cat "$O/probe.json"
done
