#!/bin/bash
# round 4, call 18: sparse kernel prefetches on top of SPARSE_AADPF (product): the combination's power under the tail
# (hppf), the H^64 basis before the counter-mode constants (basispf); c4s, same box, alternating twice; then c4 / c3 / c2 of
# the product against the DPP-only build (the sparse kernel is not on their path: a check that nothing else moved)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c18; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
for k in 1 2; do
  for n in aadpf2 hppf basispf; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
