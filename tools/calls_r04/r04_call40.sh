#!/bin/bash
# round 4, call 40: the sparse kernel's queued tail fraction on the final kernel: the last 1/2, 1/3 or 1/4 (product) of the
# records from the launch's queue, c4s, same box, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c40; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
for k in 1 2; do
  for n in t4 t3 t2; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s --clock $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-330
  done
done
