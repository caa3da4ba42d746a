#!/bin/bash
# plugin path on mapped staging: parity (full GPU suite) + ptlsbench-shape timing; mapped-transport slice sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "plugin:200:python -c 'import sys; sys.path[:0]=[\"tests\",\"hsig-picotls_amd\"]; import torch; torch.cuda.init(); import bench, json; print(json.dumps(bench.plugin_ptlsbench()))'" \
  "sweep:700:tools/r02_call18.sh"
