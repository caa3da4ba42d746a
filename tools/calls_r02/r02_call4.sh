#!/bin/bash
# round-2 evidence call: host-memory transport probe, c4s sparse-kernel ablations and counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
V=hsig-picotls_amd/variants
tools/gpu_steps.sh \
  "hostmem:300:python tools/hostmem_probe.py" \
  "c4s_ablate:300:python tools/time_cfg.py --config c4s hsig-picotls_amd/libptls_hip.so $V/libptls_hip_sab1.so $V/libptls_hip_sab2.so $V/libptls_hip_sab3.so" \
  "c4s_pmc:800:tools/pmc_passes.sh gpurun_out/pmc_c4s --config c4s --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-plugin && python3 tools/pmc_summary.py gpurun_out/pmc_c4s --json gpurun_out/lds_c4s.json"
