#!/bin/bash
# round 3, call 11: windowed lane combination (gf_mul_win4) + worker with inline records and pipelined polls:
# GPU suite (worker off, then on), c4s A/B against the bit-serial combination (ab/cur/libptls_hip_win0.so), plugin latency
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c11; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -x -v --timeout 250 --timeout-method thread > "$O/worker.log" 2>&1 \
  || { echo "worker rc=$?"; tail -40 "$O/worker.log"; exit 1; }
tail -2 "$O/worker.log"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
PTLS_HIP_PLUGIN_WORKER=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_worker.log" 2>&1 \
  || { echo "pytest worker rc=$?"; tail -40 "$O/pytest_worker.log"; exit 1; }
tail -2 "$O/pytest_worker.log"
P=hsig-picotls_amd/libptls_hip.so; V=ab/cur/libptls_hip_win0.so
for rep in 1 2; do
  for L in $P $V; do
    timeout -k 10 180 python tools/time_cfg.py $R/$L --config c4s --reps 11 >> "$O/ab.log" 2>&1 || { echo "time_cfg rc=$?"; tail "$O/ab.log"; exit 1; }
  done
done
grep -v amdgpu.ids "$O/ab.log"
for W in 1 0 1 0; do
  echo "worker=$W" >> "$O/plugin.log"
  PTLS_HIP_PLUGIN_WORKER=$W timeout -k 10 120 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; tail "$O/plugin.log"; exit 1; }
done
echo "win0 worker=0" >> "$O/plugin.log"
PTLS_HIP_LIB=$R/$V PTLS_HIP_PLUGIN_WORKER=0 timeout -k 10 120 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; exit 1; }
grep -v amdgpu.ids "$O/plugin.log"
