#!/bin/bash
# round 5, call 23: seal folds the stretch's last two ciphertext blocks into the first generic pair's AES (ctr_ghash
# with HASH) instead of two dependent multiplies after the stretch: GPU suite, base (variants/libptls_hip_base.so = the
# previous product) vs new alternating on c3 / c4 / c2, and the task-phase stamps of the new code on c3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c23; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; B=$V/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so; K=$V/libptls_hip_ksstamps.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for c in c3 c4 c2; do
  timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N $B $N --config $c 2>&1 | grep GiB || exit 1
done > "$O/ab.log"
cat "$O/ab.log"
timeout -k 10 200 python -u tools/keyswitch_stamps.py $K --config c3 2>&1 | grep -v amdgpu.ids > "$O/phases.log" && cat "$O/phases.log"
