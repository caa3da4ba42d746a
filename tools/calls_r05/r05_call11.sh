#!/bin/bash
# round 5, call 11: lanes per record against batch size (a 1 GiB c2-shape seal took 1.06-1.12 ms
# against the 0.82 the bench rate predicts).  c2's 16 KiB records and c3's 1350 B records at several batch sizes,
# every lanes-per-record value the planner could take, the product library timed twice per point.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c11; mkdir -p "$O"
L=$R/hsig-picotls_amd/libptls_hip.so
for n in 4096 16384 65536 262144; do
  for g in 4 8 16 32; do
    echo "c2 records=$n lanes=$g"
    timeout -k 10 120 python -u tools/time_cfg.py $L $L --config c2 --records $n --lanes $g 2>&1 | grep GiB || exit 1
  done
done > "$O/c2_sizes.log"
cat "$O/c2_sizes.log"
for n in 65536 262144 786432; do
  for g in 2 4 8; do
    echo "c3 records=$n lanes=$g"
    timeout -k 10 120 python -u tools/time_cfg.py $L $L --config c3 --records $n --lanes $g 2>&1 | grep GiB || exit 1
  done
done > "$O/c3_sizes.log"
cat "$O/c3_sizes.log"
