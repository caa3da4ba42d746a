#!/bin/bash
# PIPE_KEYS=1 (early keystream pass of the next key run's shortest tasks): parity (variant cases + bench c4's full
# open check and golden records), then same-box A/B timing on c4 against the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; V=hsig-picotls_amd/variants/libptls_hip_pipe.so
tools/gpu_steps.sh \
  "vcase:400:PTLS_HIP_LIB=$V python tests/variant_case.py" \
  "bench_c4:300:PTLS_HIP_LIB=$V python bench.py --config c4 --no-cpu-baseline --no-e2e --no-plugin" \
  "ab_c4:300:python tools/time_cfg.py $P $V $P $V --config c4" \
  "ab_c4u:300:python tools/time_cfg.py $P $V --config c4 --fixed-len 8224"
