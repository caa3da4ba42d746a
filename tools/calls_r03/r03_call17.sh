#!/bin/bash
# round 3, call 17: the lanes-per-record crossover after the G = 32 window combination: configs[3]'s lengths with 64, 96, 128
# and 192 records per key (4M records, 65536 / 43690 / 32768 / 21845 keys) at 8 / 16 / 32 lanes, seal+open
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c17; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so
for K in 65536 43690 32768 21845; do
  for G in 8 16 32; do
    echo "keys=$K" >> "$O/cross.log"
    timeout -k 10 200 python tools/time_cfg.py $P --config c4 --keys $K --lanes $G --reps 5 >> "$O/cross.log" 2>&1 || { echo "rc=$?"; tail "$O/cross.log"; exit 1; }
  done
done
grep -v amdgpu.ids "$O/cross.log"
