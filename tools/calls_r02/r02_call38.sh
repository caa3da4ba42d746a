#!/bin/bash
# mapped pipeline: first slices ramp up (1/16, 1/4) so slice 0's planning is short (O = no ramp, P = ramp), A/B/A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=hsig-picotls_amd/variants/libptls_hip_noramp.so
steps=("ptests:400:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'pipeline or tls13 or empty or supp'")
for c in c3 c4 c2; do
  steps+=("${c}_o1:200:PTLS_HIP_LIB=$O python tools/transport_mix_probe.py $c 0" "${c}_p1:200:python tools/transport_mix_probe.py $c 0"
          "${c}_o2:200:PTLS_HIP_LIB=$O python tools/transport_mix_probe.py $c 0" "${c}_p2:200:python tools/transport_mix_probe.py $c 0")
done
tools/gpu_steps.sh "${steps[@]}"
