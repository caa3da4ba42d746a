#!/bin/bash
# host-resident transports at the same time: MAPPED (CU-initiated PCIe) for part of the batch, COPY (SDMA) for the rest
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_steps.sh "mix_c2:300:python tools/transport_mix_probe.py c2" "mix_c3:300:python tools/transport_mix_probe.py c3"
