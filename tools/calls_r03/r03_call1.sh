#!/bin/bash
# round 3, call 1: same-box A/B of c2: the round-1 tree (678d06d), the round-2 tree (890b6c1) and
# HEAD, alternating x2 (tools/time_cfg.py, random records), then kernel cycles per launch of each (GRBM_GUI_ACTIVE, PMC
# pass per library), then the GPU test suite and one default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c1; mkdir -p "$O"
LIBS=(ab/r01/hsig-picotls_amd/libptls_hip.so ab/r02/hsig-picotls_amd/libptls_hip.so hsig-picotls_amd/libptls_hip.so)
for rep in 1 2; do
  for L in "${LIBS[@]}"; do
    timeout -k 10 180 python tools/time_cfg.py "$L" --config c2 --clock --reps 11 >> "$O/ab.log" 2>&1 || { echo "time_cfg $L rc=$?"; exit 1; }
  done
done
cat "$O/ab.log"
i=0
for L in "${LIBS[@]}"; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES -T --output-format csv \
      -d "$O/pmc$i" -o run -- python3 "$R/tools/time_cfg.py" "$R/$L" --config c2 --reps 4 > "$O/pmc$i.log" 2>&1) \
      || { echo "pmc $L rc=$?"; exit 1; }
  i=$((i+1))
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
  || { echo "pytest rc=$?"; tail -30 "$O/pytest.log"; exit 1; }
tail -3 "$O/pytest.log"
timeout -k 10 600 python bench.py > "$O/bench_c2.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench_c2.log"; exit 1; }
tail -1 "$O/bench_c2.log"
