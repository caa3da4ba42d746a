#!/bin/bash
# host-resident pipeline planning: counting sort + caller-order descriptors when the plan keeps the order
# (O = engine before both, P = current), A/B/A/B, mapped transport only; pipeline parity tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=hsig-picotls_amd/variants/libptls_hip_engold.so
steps=("ptests:400:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'pipeline or tls13 or sparse or mixed or empty or supp'")
for c in c3 c4 c2; do
  steps+=("${c}_o1:200:PTLS_HIP_LIB=$O python tools/transport_mix_probe.py $c 0" "${c}_p1:200:python tools/transport_mix_probe.py $c 0"
          "${c}_o2:200:PTLS_HIP_LIB=$O python tools/transport_mix_probe.py $c 0" "${c}_p2:200:python tools/transport_mix_probe.py $c 0")
done
tools/gpu_steps.sh "${steps[@]}"
