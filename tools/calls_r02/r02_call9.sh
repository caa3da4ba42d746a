#!/bin/bash
# G = 32 lanes per record and the GEN_MASK generic-path variant: parity, then c4 / c3 / c2 timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; M=hsig-picotls_amd/variants/libptls_hip_gmask.so
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "c4_16:300:python tools/time_cfg.py --config c4 --lanes 16 $P $M $P $M" \
  "c4_32:300:python tools/time_cfg.py --config c4 --lanes 32 $P $M $P $M" \
  "c3:300:python tools/time_cfg.py --config c3 $P $M $P $M" \
  "c2:300:python tools/time_cfg.py --config c2 $P $M $P $M"
