#!/bin/bash
# round 3, call 6: sparse kernel with per-lane stretch starts (no generic head) and the single-record table build left
# to waves 1-3; GPU suite; A/B against the round-2 tree on c2 / c3 / c4s; plugin latency; phase stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c6; mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
R2=ab/r02/hsig-picotls_amd/libptls_hip.so; P=hsig-picotls_amd/libptls_hip.so
for rep in 1 2; do
  for L in $R2 $P; do
    timeout -k 10 240 python tools/time_cfg.py $L --config c4s --reps 11 >> "$O/ab.log" 2>&1 || exit 1
    timeout -k 10 240 python tools/time_cfg.py $L --config c3 --reps 6 >> "$O/ab.log" 2>&1 || exit 1
    timeout -k 10 240 python tools/time_cfg.py $L --config c2 --reps 6 >> "$O/ab.log" 2>&1 || exit 1
  done
done
grep -v amdgpu.ids "$O/ab.log"
timeout -k 10 300 python tools/sparse_stamps.py > "$O/sparse_stamps.log" 2>&1 || { echo "sparse stamps rc=$?"; tail -20 "$O/sparse_stamps.log"; exit 1; }
tail -1 "$O/sparse_stamps.log"
timeout -k 10 300 python tools/plugin_stamps.py > "$O/stamps.log" 2>&1 || { echo "stamps rc=$?"; tail -20 "$O/stamps.log"; exit 1; }
tail -1 "$O/stamps.log"
for rep in 1 2; do
  for L in $R2 $P; do
    echo "lib=$L" >> "$O/plugin.log"
    PTLS_HIP_LIB=$R/$L timeout -k 10 300 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; exit 1; }
  done
done
grep -v amdgpu.ids "$O/plugin.log"
