#!/bin/bash
# same-box A/B of the sparse kernel change (O = previous commit's sparse_kernel.hip, P = current)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; O=hsig-picotls_amd/variants/libptls_hip_spold.so
tools/gpu_steps.sh \
  "ab_c4s:200:python tools/time_cfg.py $O $P $O $P $O $P --config c4s" \
  "ab_c4s_short:200:python tools/time_cfg.py $O $P $O $P --config c4s --fixed-len 1350" \
  "ab_probe_old:120:PTLS_HIP_LIB=$O python tools/plugin_probe.py" \
  "ab_probe_new:120:python tools/plugin_probe.py"
