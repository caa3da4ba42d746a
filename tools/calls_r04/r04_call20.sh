#!/bin/bash
# round 4, call 20: batch kernel loads a task's first AAD block before the counter-mode constants (BATCH_AADPF): GPU suite,
# then same-box A/B against the previous product (aadpf2) on c3, c4, c2, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c20; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for c in c3 c4 c2; do
  for n in aadpf2 baadpf aadpf2 baadpf; do
    timeout -k 10 200 python -u tools/time_cfg.py --config $c $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
