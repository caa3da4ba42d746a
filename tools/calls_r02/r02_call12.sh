#!/bin/bash
# planner crossover: records per key 8..64 on configs[3]'s shape (AES-256, 64 B - 16 KiB, 64K keys), lanes 16 / 32 / sparse
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so
steps=()
for per in 8 16 24 32 48; do
  n=$((per * 65536))
  for l in 16 32 64; do
    steps+=("per${per}_l${l}:300:python tools/time_cfg.py --config c4 --records $n --lanes $l $P")
  done
done
tools/gpu_steps.sh "${steps[@]}"
