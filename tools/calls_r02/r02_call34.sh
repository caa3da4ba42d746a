#!/bin/bash
# round-end evidence refresh (part 2): c4, c4s, then the plugin path's kernel trace (tools/plugin_trace_summary.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 1000 tools/refresh_profiles.sh r02 c4 c4s && \
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/plugprof3" -o plug -- python3 "$GRAFT_REPO_ROOT/tools/plugin_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/plugprof3.log" 2>&1 && echo "plugin trace ok"
