#!/bin/bash
# round 3, call 26: long single records on two waves at stride 128 (H^128 basis plane): size sweep (incl. 2-16 KiB records)
# and worker lifecycle first, then the GPU suite, plugin latency on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c26; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_plugin_sizes.py tests/test_gpu_worker.py -x -v --timeout 300 --timeout-method thread > "$O/sizes.log" 2>&1 \
  || { echo "sizes rc=$?"; tail -40 "$O/sizes.log"; exit 1; }
tail -1 "$O/sizes.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for W in 1 0 1; do
  echo "worker=$W" >> "$O/plugin.log"
  PTLS_HIP_PLUGIN_WORKER=$W timeout -k 10 120 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; tail "$O/plugin.log"; exit 1; }
done
grep -v amdgpu.ids "$O/plugin.log"
for rep in 1 2; do
  timeout -k 10 200 python tools/time_cfg.py $R/hsig-picotls_amd/libptls_hip.so --config c4s --reps 11 >> "$O/c4s.log" 2>&1 || { echo "rc=$?"; exit 1; }
done
grep -v amdgpu.ids "$O/c4s.log"
