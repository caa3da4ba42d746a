#!/bin/bash
# host NUMA placement of the zero-copy host-resident path (tools/numa_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_steps.sh "numa:400:python tools/numa_probe.py"
