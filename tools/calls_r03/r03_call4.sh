#!/bin/bash
# round 3, call 4: split tasks with one B per task (from its shortest record): parity, then same-box c4 A/B against
# the no-split build (variants/libptls_hip_nosplit.so: SPLIT_TASKS=0, no spill) and split thresholds; plugin latency
# with coherent vs default staging
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c4; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_dealing.py -x -q --timeout 300 --timeout-method thread \
  > "$O/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
P=hsig-picotls_amd/libptls_hip.so; NS=hsig-picotls_amd/variants/libptls_hip_nosplit.so
for rep in 1 2; do
  timeout -k 10 240 python tools/time_cfg.py $NS --config c4 --clock --reps 6 >> "$O/split_c4.log" 2>&1 || exit 1
  for pct in 0 75 100 150; do
    echo "PTLS_HIP_SPLIT_PCT=$pct" >> "$O/split_c4.log"
    PTLS_HIP_SPLIT_PCT=$pct timeout -k 10 240 python tools/time_cfg.py $P --config c4 --clock --reps 6 >> "$O/split_c4.log" 2>&1 || exit 1
  done
done
grep -v amdgpu.ids "$O/split_c4.log"
for st in coherent default coherent default; do
  echo "staging=$st" >> "$O/plugin.log"
  PTLS_HIP_PLUGIN_STAGING=$st timeout -k 10 300 python tools/plugin_probe.py >> "$O/plugin.log" 2>&1 || { echo "plugin rc=$?"; exit 1; }
done
grep -v amdgpu.ids "$O/plugin.log"
