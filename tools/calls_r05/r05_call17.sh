#!/bin/bash
# round 5, call 17: where the batch kernel's wave time goes inside tasks (KS_STAMPS diagnostic build with the task-phase
# marks, variants/libptls_hip_ksstamps.so; tools/keyswitch_stamps.py), c2 / c3 / c4, and the stamp build's own cost on c3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c17; mkdir -p "$O"
K=$R/hsig-picotls_amd/variants/libptls_hip_ksstamps.so; N=$R/hsig-picotls_amd/libptls_hip.so
for c in c2 c3 c4; do
  timeout -k 10 200 python -u tools/keyswitch_stamps.py $K --config $c 2>&1 | grep -v amdgpu.ids || exit 1
done > "$O/phases.log"
cat "$O/phases.log"
timeout -k 10 200 python -u tools/time_cfg.py $N $K --config c3 2>&1 | grep GiB > "$O/stamp_cost_c3.log" && cat "$O/stamp_cost_c3.log"
