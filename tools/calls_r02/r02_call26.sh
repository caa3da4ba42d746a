#!/bin/bash
# AES tables built with batched T0 loads and b128 stores: full GPU suite, plugin latency, batch-kernel timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "probe:120:python tools/plugin_probe.py" \
  "t_c2:200:python tools/time_cfg.py $P $P --config c2" \
  "t_c3:200:python tools/time_cfg.py $P $P --config c3" \
  "t_c4:200:python tools/time_cfg.py $P $P --config c4" \
  "t_c4s:200:python tools/time_cfg.py $P $P --config c4s" \
  "t_small:200:python tools/time_cfg.py $P $P --config c3 --records 32768"
