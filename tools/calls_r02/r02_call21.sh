#!/bin/bash
# CTRHI_PROBE upper bound: rounds 1-2 of the skewed loop with the counter's high byte taken as fixed (1 + 4 lookups
# instead of 2 + 8 per block; wrong output, timing only), against the product build, alternating A/B/A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; V=hsig-picotls_amd/variants/libptls_hip_ctrhi.so
tools/gpu_steps.sh \
  "c2:200:python tools/time_cfg.py $P $V $P $V --config c2" \
  "c3:200:python tools/time_cfg.py $P $V $P $V --config c3" \
  "c4:300:python tools/time_cfg.py $P $V $P $V --config c4"
