#!/bin/bash
# final verification of the round's build: full GPU suite, smoke, default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:400:python bench.py"
