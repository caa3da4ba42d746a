#!/bin/bash
# round 4, call 17: sparse kernel record-setup prefetches (SPARSE_AADPF / SPARSE_TAGPF variants) against the DPP build on
# c4s, same box, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c17; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
for k in 1 2; do
  for n in dpp aadpf tagpf aadtagpf; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
