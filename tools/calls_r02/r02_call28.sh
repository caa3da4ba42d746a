#!/bin/bash
# sparse kernel: one generic range without a stretch, H^64 basis loads before the counter-mode constants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "probe:120:python tools/plugin_probe.py" \
  "t_c4s:200:python tools/time_cfg.py $P $P $P --config c4s" \
  "t_c4s_short:200:python tools/time_cfg.py $P $P --config c4s --fixed-len 1350"
