#!/bin/bash
# round 4, call 34: the sparse batch kernel's lane combination with 8 lookups in flight (SPARSE_WIN_LB = 8, no more scratch
# than 4 after the spill fix) against the product (nospill), c4s, same box, alternating three times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c34; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
for k in 1 2 3; do
  for n in nospill lb8; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
