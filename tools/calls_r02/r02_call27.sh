#!/bin/bash
# plugin completion words on the AEAD and single-block ECB paths: full GPU suite, plugin and ECB per-call latency
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
P=hsig-picotls_amd/libptls_hip.so
tools/gpu_steps.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "probe:120:python tools/plugin_probe.py"
