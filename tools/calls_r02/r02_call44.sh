#!/bin/bash
# planner re-check on the final build: lanes per record for c3 / c2 / c4 (same box, two alternations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so
steps=()
for l in 2 4 8 2 4 8; do steps+=("c3_g$l:120:python tools/time_cfg.py $P --config c3 --lanes $l"); done
for l in 4 8 16 4 8 16; do steps+=("c2_g$l:120:python tools/time_cfg.py $P --config c2 --lanes $l"); done
for l in 16 32 16 32; do steps+=("c4_g$l:200:python tools/time_cfg.py $P --config c4 --lanes $l"); done
tools/gpu_steps.sh "${steps[@]}"
