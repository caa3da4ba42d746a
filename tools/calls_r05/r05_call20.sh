#!/bin/bash
# round 5, call 20: sub-phases of the generic elements after the stretch (KS_STAMPS build with marks inside
# generic_pair: loads issued, AES, finish, GHASH), c3 and c4; and the product with generic_pair's finish-then-GHASH order
# (base = the previous product) on c3 / c4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c20; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; K=$V/libptls_hip_ksstamps.so; B=$V/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
for c in c3 c4; do
  timeout -k 10 200 python -u tools/keyswitch_stamps.py $K --config $c 2>&1 | grep -v amdgpu.ids || exit 1
done > "$O/phases.log"
cat "$O/phases.log"
for c in c3 c4; do
  timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config $c 2>&1 | grep GiB || exit 1
done > "$O/ab.log"
cat "$O/ab.log"
