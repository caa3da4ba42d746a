#!/bin/bash
# round 5, call 14: why a 1 GiB c2-shape launch runs ~20 % below the 16 GiB one at every lanes-per-record value (call 11):
# in-run clock, workgroup start / end spread and span from the kernels' own stamps (time_cfg --clock), at 1, 4 and 16 GiB
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c14; mkdir -p "$O"
N=$R/hsig-picotls_amd/libptls_hip.so
for n in 65536 262144 0; do
  extra=""; [ $n != 0 ] && extra="--records $n"
  echo "== c2 records=$n"
  timeout -k 10 200 python -u tools/time_cfg.py $N $N --config c2 $extra --clock 2>&1 | grep GiB || exit 1
done > "$O/clock_by_size.log"
cat "$O/clock_by_size.log"
