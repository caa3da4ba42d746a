#!/bin/bash
# round 3, call 21: sparse kernel with every lane-derived value computed per record (scratch 84 -> 24 B per lane, one 16-B
# reload per record): GPU suite, c4s timing, c4s HBM traffic (tools/profile_round.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c21; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for rep in 1 2; do
  timeout -k 10 200 python tools/time_cfg.py $R/hsig-picotls_amd/libptls_hip.so --config c4s --reps 11 >> "$O/c4s.log" 2>&1 || { echo "rc=$?"; exit 1; }
done
grep -v amdgpu.ids "$O/c4s.log"
bash tools/profile_round.sh r03b c4s > "$O/traffic.log" 2>&1 || { echo "profile rc=$?"; tail "$O/traffic.log"; exit 1; }
grep -E "traffic_over|fetch_bytes_per|write_bytes_per|bench_seal" "$O/traffic.log"
