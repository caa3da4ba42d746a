#!/bin/bash
# round 5, call 19: EXPERIMENT, wave stagger after the first key switch (batch_kernel.h STAGGER = 1 / 3: wave w waits
# w x ~4 / ~12 us) so that waves running identical tasks (c3's uniform records) do not reach their generic phases
# together; base vs stag1 vs stag3 alternating on c3, c2, c4; the stamped phase shares of stag3 on c3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c19; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; B=$V/libptls_hip_base.so; S1=$V/libptls_hip_stag1.so; S3=$V/libptls_hip_stag3.so
for c in c3 c2 c4; do
  timeout -k 10 300 python -u tools/time_cfg.py $B $S1 $S3 $B $S1 $S3 --config $c --clock 2>&1 | grep GiB || exit 1
done > "$O/ab.log"
cut -c1-200 "$O/ab.log"
