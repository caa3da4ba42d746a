#!/bin/bash
# round 3, call 24: planner checks after the round's kernel changes: c4 at G = 32 with 512- vs 768-thread workgroups, and
# configs[3]'s lengths at 16 / 24 records per key with G = 32 against the sparse kernel (64), alternating x2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c24; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so
for rep in 1 2; do
  for W in 768 512; do
    timeout -k 10 200 python tools/time_cfg.py $P --config c4 --lanes 32 --wg $W --reps 5 >> "$O/plan.log" 2>&1 || { echo "rc=$?"; tail "$O/plan.log"; exit 1; }
  done
  for K in 262144 174762; do
    for G in 32 64; do
      echo "keys=$K" >> "$O/plan.log"
      timeout -k 10 200 python tools/time_cfg.py $P --config c4 --keys $K --lanes $G --reps 5 >> "$O/plan.log" 2>&1 || { echo "rc=$?"; tail "$O/plan.log"; exit 1; }
    done
  done
done
grep -v amdgpu.ids "$O/plan.log"
