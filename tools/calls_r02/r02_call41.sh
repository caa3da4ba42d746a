#!/bin/bash
# mapped pipeline slice size after the planning change (slice MiB x 4 = the mapped slice), c3 / c4 / c2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
steps=()
for c in c3 c4 c2; do for m in 16 32 64 128; do steps+=("${c}_${m}:200:python tools/transport_mix_probe.py $c 0 $m"); done; done
tools/gpu_steps.sh "${steps[@]}"
