#!/bin/bash
# round 4, call 32: sparse kernel without its per-record scratch reloads (the lane index by a volatile mbcnt, the window
# table's zero entry from an opaque zero): GPU suite, c4s A/B against the previous product (prod), alternating twice, plugin probe
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c32; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for k in 1 2; do
  for n in prod nospill; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
for n in prod nospill; do
  PTLS_HIP_LIB=$V/libptls_hip_$n.so timeout -k 10 120 python -u tools/plugin_probe.py > "$O/probe_$n.json" 2>/dev/null && echo "$n $(cat $O/probe_$n.json | cut -c1-600)" || exit 1
done
