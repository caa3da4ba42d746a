#!/bin/bash
# round 4, call 19: GPU suite on the product (DPP reductions + SPARSE_AADPF); c4s A/B of the next-record touch prefetch
# (SPARSE_NEXTPF variant) against it, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c19; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for k in 1 2; do
  for L in $R/hsig-picotls_amd/libptls_hip.so $V/libptls_hip_nextpf.so; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s $L > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
