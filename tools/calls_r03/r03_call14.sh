#!/bin/bash
# round 3, call 14 (second run, the call-13 build: the first run of this call on a build with constant-space key pointers and worker ECB requests faulted in the lifecycle test, reverted); worker + size sweep; plugin latency; c3 HBM traffic with records at 16- and
# 128-byte aligned offsets (PTLS_BENCH_ALIGN), each pass under its own limit (tools/profile_round.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c14; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_plugin_sizes.py tests/test_gpu_worker.py -x -v --timeout 300 --timeout-method thread > "$O/sizes.log" 2>&1 \
  || { echo "sizes rc=$?"; tail -40 "$O/sizes.log"; exit 1; }
tail -1 "$O/sizes.log"
for W in 1 0; do
  echo "worker=$W" >> "$O/plugin.log"
  PTLS_HIP_PLUGIN_WORKER=$W timeout -k 10 120 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; tail "$O/plugin.log"; exit 1; }
done
grep -v amdgpu.ids "$O/plugin.log"
for A in 16 128; do
  PTLS_BENCH_ALIGN=$A bash tools/profile_round.sh a$A c3 > "$O/traffic_a$A.log" 2>&1 || { echo "profile a$A rc=$?"; tail "$O/traffic_a$A.log"; exit 1; }
  grep -E "traffic_over|fetch_bytes_per|write_bytes_per|bench_seal" "$O/traffic_a$A.log"
done
timeout -k 10 200 python tools/worker_stamps.py > "$O/wstamps.log" 2>&1 || { echo "wstamps rc=$?"; tail "$O/wstamps.log"; exit 1; }
grep -v amdgpu.ids "$O/wstamps.log"
