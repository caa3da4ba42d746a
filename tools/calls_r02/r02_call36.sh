#!/bin/bash
# host-resident pipeline planning: counting sort of the sparse-kernel slices (O = previous engine, P = current);
# pipeline parity tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=hsig-picotls_amd/variants/libptls_hip_engold.so
tools/gpu_steps.sh \
  "ptests:400:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k 'pipeline or tls13 or sparse or mixed or empty'" \
  "mix_c3_old:300:PTLS_HIP_LIB=$O python tools/transport_mix_probe.py c3 0,1" \
  "mix_c3_new:300:python tools/transport_mix_probe.py c3 0,1" \
  "mix_c4_old:300:PTLS_HIP_LIB=$O python tools/transport_mix_probe.py c4 0,1" \
  "mix_c4_new:300:python tools/transport_mix_probe.py c4 0,1"
