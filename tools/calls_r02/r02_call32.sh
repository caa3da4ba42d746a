#!/bin/bash
# bound on c4's key-switch cost under dynamic dealing: key switches after the first neither wait nor rebuild, the task
# counter runs on across keys (timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; D=hsig-picotls_amd/variants/libptls_hip_dynnobar.so
tools/gpu_steps.sh \
  "kd_c4:300:python tools/time_cfg.py $P $D $P $D --config c4 --lanes 16" \
  "kd_c4g8:300:python tools/time_cfg.py $P $D --config c4 --lanes 8" \
  "kd_c4u:300:python tools/time_cfg.py $P $D --config c4 --lanes 16 --fixed-len 8224"
