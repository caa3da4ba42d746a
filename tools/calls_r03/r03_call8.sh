#!/bin/bash
# round 3, call 8: the resident plugin worker (tests/test_gpu_worker.py first, then the full GPU suite), plugin latency
# A/B: worker / one launch per call (PTLS_HIP_PLUGIN_WORKER=0) / the round-2 tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c8; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -x -v --timeout 250 --timeout-method thread > "$O/worker.log" 2>&1 \
  || { echo "worker rc=$?"; tail -60 "$O/worker.log"; exit 1; }
tail -3 "$O/worker.log"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
R2=ab/r02/hsig-picotls_amd/libptls_hip.so; P=hsig-picotls_amd/libptls_hip.so
for rep in 1 2; do
  for W in 1 0; do
    echo "lib=$P worker=$W" >> "$O/plugin.log"
    PTLS_HIP_PLUGIN_WORKER=$W PTLS_HIP_LIB=$R/$P timeout -k 10 300 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; tail "$O/plugin.log"; exit 1; }
  done
  echo "lib=$R2" >> "$O/plugin.log"
  PTLS_HIP_LIB=$R/$R2 timeout -k 10 300 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; exit 1; }
done
grep -v amdgpu.ids "$O/plugin.log"
