#!/bin/bash
# round 5, call 21: generic data blocks as one 16-byte load of the bytes ending at the block's end (batch_kernel.h
# tail_load / tail_shift; the loads no longer wait inside divergent branches before the element pair's AES; variants/
# libptls_hip_tail.so) and, in the product, also the AAD block without branches (load_block_nb: one wait): GPU suite,
# base (variants/libptls_hip_base.so = the previous product) vs tail vs new alternating on c3 / c4 / c2 / c3 packed at
# 16 and 1 bytes, then the task-phase stamps of the new code on c3 / c4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c21; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; B=$V/libptls_hip_base.so; T=$V/libptls_hip_tail.so; N=$R/hsig-picotls_amd/libptls_hip.so
K=$V/libptls_hip_ksstamps.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for c in c3 c4 c2; do
  timeout -k 10 300 python -u tools/time_cfg.py $B $T $N $B $T $N --config $c 2>&1 | grep GiB || exit 1
done > "$O/ab.log"
for a in 16 1; do
  echo "c3 align $a"
  PTLS_BENCH_ALIGN=$a timeout -k 10 300 python -u tools/time_cfg.py $B $T $N $B $T $N --config c3 2>&1 | grep GiB || exit 1
done >> "$O/ab.log"
cat "$O/ab.log"
for c in c3 c4; do
  timeout -k 10 200 python -u tools/keyswitch_stamps.py $K --config $c 2>&1 | grep -v amdgpu.ids || exit 1
done > "$O/phases.log"
cat "$O/phases.log"
