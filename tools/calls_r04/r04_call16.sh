#!/bin/bash
# round 4, call 16: cross-lane reductions on the VALU (DPP + permlane swaps instead of ds_bpermute): GPU suite on the new
# build, then same-box A/B (base = HEAD's library, dpp = this build) on c4s, c4, c3, c2, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c16; mkdir -p "$O"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
B=$R/hsig-picotls_amd/variants/libptls_hip_base.so; D=$R/hsig-picotls_amd/variants/libptls_hip_dpp.so
for c in c4s c4 c3 c2; do
  for L in $B $D $B $D; do
    timeout -k 10 200 python -u tools/time_cfg.py --config $c --clock $L > "$O/ab_$c.log" 2>&1 || { cat "$O/ab_$c.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab_$c.log" | cut -c1-240
  done
done
