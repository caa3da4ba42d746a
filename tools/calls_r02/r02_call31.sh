#!/bin/bash
# bound on c4's key-switch waits: static dealing with and without the barriers / table rebuilds of later key switches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; S=hsig-picotls_amd/variants/libptls_hip_static.so; N=hsig-picotls_amd/variants/libptls_hip_nobar.so
tools/gpu_steps.sh \
  "ks_c4:300:python tools/time_cfg.py $P $S $N $P $S $N --config c4 --lanes 16" \
  "ks_c4u:300:python tools/time_cfg.py $P $S $N --config c4 --lanes 16 --fixed-len 8224"
