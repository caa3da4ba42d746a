#!/bin/bash
# where c4's time goes: AES-only / GHASH-only probes at 16 and 32 lanes, and c4's shape with one factor changed at a time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; V=hsig-picotls_amd/variants
tools/gpu_steps.sh \
  "c4_16:300:python tools/time_cfg.py --config c4 --lanes 16 $P $V/libptls_hip_split1.so $V/libptls_hip_split2.so" \
  "c4_32:300:python tools/time_cfg.py --config c4 --lanes 32 $P $V/libptls_hip_split1.so $V/libptls_hip_split2.so" \
  "c4_fixed:300:python tools/time_cfg.py --config c4 --lanes 16 --fixed-len 8224 $P" \
  "c4_1key_fixed:300:python tools/time_cfg.py --config c4 --keys 1 --fixed-len 8224 $P" \
  "c4_1key_mixed:300:python tools/time_cfg.py --config c4 --keys 1 $P" \
  "c2_aes256:300:python tools/time_cfg.py --config c2 --key-len 32 $P"
