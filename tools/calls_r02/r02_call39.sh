#!/bin/bash
# final build: full GPU suite, smoke, and the four full bench lines (host_e2e after the planning change)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2:400:python bench.py --config c2 > gpurun_out/bench_c2_full.log 2>&1" \
  "bench_c3:400:python bench.py --config c3 > gpurun_out/bench_c3_full.log 2>&1" \
  "bench_c4:400:python bench.py --config c4 > gpurun_out/bench_c4_full.log 2>&1" \
  "bench_c4s:400:python bench.py --config c4s > gpurun_out/bench_c4s_full.log 2>&1"
