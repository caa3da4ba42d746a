#!/bin/bash
# round 3, call 10 (re-entry after the container was re-created): the plugin worker's lifecycle test, the full GPU suite,
# plugin latency with the worker on / off, one default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c10; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py -x -v --timeout 250 --timeout-method thread > "$O/worker.log" 2>&1 \
  || { echo "worker rc=$?"; tail -60 "$O/worker.log"; exit 1; }
tail -3 "$O/worker.log"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for W in 1 0 1 0; do
  echo "worker=$W" >> "$O/plugin.log"
  PTLS_HIP_PLUGIN_WORKER=$W timeout -k 10 120 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; tail "$O/plugin.log"; exit 1; }
done
grep -v amdgpu.ids "$O/plugin.log"
timeout -k 10 300 python bench.py > "$O/bench_c2.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench_c2.log"; exit 1; }
tail -1 "$O/bench_c2.log" | cut -c1-600
