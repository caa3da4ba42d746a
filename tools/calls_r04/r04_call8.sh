#!/bin/bash
# round 4, call 8 (after call 7's fault was traced to a sign-extended readfirstlane in the pointer
# rebuild): the constant-address-space worker with the fix, through the worker / size / parity tests ONCE; then per-call
# latency: shipping worker (vector key loads, ECB through the worker), the same with one launch per ECB block, and the
# constant-address-space worker
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c8; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so; W=$R/hsig-picotls_amd/variants/libptls_hip_wconst.so
PTLS_HIP_LIB=$W timeout -k 10 500 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_plugin_sizes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/wconst_tests.log" 2>&1
rc=$?; tail -3 "$O/wconst_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/wconst_tests.log" | head; exit $rc; }
for i in 1 2; do
  PTLS_HIP_LIB=$P timeout -k 10 120 python -u tools/plugin_probe.py 2>/dev/null | sed 's/^/vector+ecbworker: /' || exit 1
  PTLS_HIP_ECB_LAUNCH=1 PTLS_HIP_LIB=$P timeout -k 10 120 python -u tools/plugin_probe.py 2>/dev/null | sed 's/^/vector+ecblaunch: /' || exit 1
  PTLS_HIP_LIB=$W timeout -k 10 120 python -u tools/plugin_probe.py 2>/dev/null | sed 's/^/scalar+ecbworker: /' || exit 1
done
