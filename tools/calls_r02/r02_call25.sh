#!/bin/bash
# plugin completion word + one-wave-per-slot key setup: the full GPU suite, then the per-call latency probe and the
# plugin path under rocprofv3 (kernel times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "probe:120:python tools/plugin_probe.py" && \
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/plugprof2" -o plug -- python3 "$GRAFT_REPO_ROOT/tools/plugin_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/plugprof2.log" 2>&1; echo "rocprof rc=$?"
