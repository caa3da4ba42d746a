#!/bin/bash
# c4 key-run balance: 64 records per key = 16 wave tasks at G = 16 for 12 waves (768 threads) or 8 waves (512)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so
tools/gpu_steps.sh \
  "g16w768:200:python tools/time_cfg.py $P $P --config c4 --lanes 16 --wg 768" \
  "g16w512:200:python tools/time_cfg.py $P $P --config c4 --lanes 16 --wg 512" \
  "g32w512:200:python tools/time_cfg.py $P $P --config c4 --lanes 32 --wg 512" \
  "g8w512:200:python tools/time_cfg.py $P $P --config c4 --lanes 8 --wg 512" \
  "u16w768:200:python tools/time_cfg.py $P --config c4 --lanes 16 --wg 768 --fixed-len 8224" \
  "u16w512:200:python tools/time_cfg.py $P --config c4 --lanes 16 --wg 512 --fixed-len 8224"
