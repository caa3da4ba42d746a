#!/bin/bash
# round 3, call 12: worker pointers as global (no flat stores): worker test, plugin latency worker on/off, worker stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c12; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -x -v --timeout 250 --timeout-method thread > "$O/worker.log" 2>&1 \
  || { echo "worker rc=$?"; tail -40 "$O/worker.log"; exit 1; }
tail -2 "$O/worker.log"
for W in 1 0 1; do
  echo "worker=$W" >> "$O/plugin.log"
  PTLS_HIP_PLUGIN_WORKER=$W timeout -k 10 120 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; tail "$O/plugin.log"; exit 1; }
done
grep -v amdgpu.ids "$O/plugin.log"
timeout -k 10 200 python tools/worker_stamps.py > "$O/wstamps.log" 2>&1 || { echo "wstamps rc=$?"; tail "$O/wstamps.log"; exit 1; }
grep -v amdgpu.ids "$O/wstamps.log"
