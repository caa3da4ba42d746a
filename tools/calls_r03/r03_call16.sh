#!/bin/bash
# round 3, call 16: G = 32 lane combination through shared per-key window tables (batch_kernel.h WINCOMB): the GPU suite,
# then c4 at 16 / 32 lanes and c4's lengths at 32 records per key, against the VALU combination (ab/cur/libptls_hip_g32valu.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c16; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
P=$R/hsig-picotls_amd/libptls_hip.so; V=$R/ab/cur/libptls_hip_g32valu.so
for rep in 1 2; do
  timeout -k 10 200 python tools/time_cfg.py $P --config c4 --lanes 16 --reps 5 >> "$O/ab.log" 2>&1 || { echo "rc=$?"; tail "$O/ab.log"; exit 1; }
  for L in $P $V; do
    timeout -k 10 200 python tools/time_cfg.py $L --config c4 --lanes 32 --reps 5 >> "$O/ab.log" 2>&1 || { echo "rc=$?"; tail "$O/ab.log"; exit 1; }
    timeout -k 10 200 python tools/time_cfg.py $L --config c4 --keys 131072 --reps 5 >> "$O/ab.log" 2>&1 || { echo "rc=$?"; tail "$O/ab.log"; exit 1; }
  done
done
grep -v amdgpu.ids "$O/ab.log"
