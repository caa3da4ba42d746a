#!/bin/bash
# sparse kernel rewrite: parity (sparse + pipeline tests), A/B timing vs the previous sparse kernel, c4s bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
V=hsig-picotls_amd/variants
tools/gpu_steps.sh \
  "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "c4s_ab:300:python tools/time_cfg.py --config c4s $V/libptls_hip_oldsparse.so hsig-picotls_amd/libptls_hip.so $V/libptls_hip_oldsparse.so hsig-picotls_amd/libptls_hip.so" \
  "c4s_1350:300:python tools/time_cfg.py --config c4s --lanes 64 --records 65536 $V/libptls_hip_oldsparse.so hsig-picotls_amd/libptls_hip.so" \
  "bench_c4s:400:python bench.py --config c4s --no-cpu-baseline --no-plugin" \
  "bench_c2:400:python bench.py --no-cpu-baseline --no-plugin"
