#!/bin/bash
# round 5, call 5: A/B of round-2 (and round-3) T-table lookups through the vector L1 instead of the LDS (GATHER_EXP,
# variants/libptls_hip_gather{1,2}.so, batch_g4 only: c2's 4 lanes per record), parity first, then alternating timing on c2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c5; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; B=$R/hsig-picotls_amd/libptls_hip.so
for v in gather1 gather2; do
  PTLS_HIP_LIB=$V/libptls_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "length_sweep and (0 or 4) or differential or large_records" \
      --timeout 200 --timeout-method thread > "$O/parity_$v.log" 2>&1 || { tail -20 "$O/parity_$v.log"; exit 1; }
  tail -1 "$O/parity_$v.log"
done
timeout -k 10 600 python -u tools/time_cfg.py $B $V/libptls_hip_gather1.so $V/libptls_hip_gather2.so $B $V/libptls_hip_gather1.so $V/libptls_hip_gather2.so \
    --config c2 > "$O/ab_c2.log" 2>&1 || { tail "$O/ab_c2.log"; exit 1; }
cat "$O/ab_c2.log"
