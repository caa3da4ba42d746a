#!/bin/bash
# plugin record: final combination through nibble tables built by idle waves (O = VALU combination, P = tables):
# plugin-path parity, per-call latency A/B, c4s batch timing unchanged
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so; O=hsig-picotls_amd/variants/libptls_hip_notree.so
tools/gpu_steps.sh \
  "ptests:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'plugin or lowlevel or iv_only or non_temporal or tls12 or aesecb or supp'" \
  "ttests:300:python -u -m pytest tests/test_gpu_tls13.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "probe_o:120:PTLS_HIP_LIB=$O python tools/plugin_probe.py" \
  "probe_p:120:python tools/plugin_probe.py" \
  "probe_o2:120:PTLS_HIP_LIB=$O python tools/plugin_probe.py" \
  "probe_p2:120:python tools/plugin_probe.py" \
  "c4s:200:python tools/time_cfg.py $O $P $O $P --config c4s"
