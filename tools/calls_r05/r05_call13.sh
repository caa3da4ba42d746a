#!/bin/bash
# round 5, call 13: c3 at 262 144 records, where call 12 read the new planner build 6 % below the base with the same lanes
# (4) and the same kernels: the same point in both orders, three alternations each, to tell order effects from the build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c13; mkdir -p "$O"
B=$R/hsig-picotls_amd/variants/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
{ echo "== order B N"; timeout -k 10 200 python -u tools/time_cfg.py $B $N $B $N $B $N --config c3 --records 262144 2>&1 | grep GiB &&
  echo "== order N B"; timeout -k 10 200 python -u tools/time_cfg.py $N $B $N $B $N $B --config c3 --records 262144 2>&1 | grep GiB; } > "$O/c3_262144.log"
cat "$O/c3_262144.log"
