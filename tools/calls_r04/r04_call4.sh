#!/bin/bash
# round 4, call 4: plugin measurements (tools/plugin_mt.py), then the chunk-queue / guided-tail A/B (c2, c3 twice)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c4; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so; V=$R/hsig-picotls_amd/variants/libptls_hip_noqueue.so
timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt.json" 2> "$O/plugin_mt.err" || { tail -20 "$O/plugin_mt.err"; exit 1; }
cat "$O/plugin_mt.json"
for c in c2 c3 c2 c3; do
  for mode in static queue guided; do
    case $mode in static) L=$V; G=1;; queue) L=$P; G=0;; guided) L=$P; G=1;; esac
    PTLS_HIP_GUIDED=$G timeout -k 10 120 python -u tools/time_cfg.py --config $c --clock $L > "$O/ab_${c}_$mode.log" 2>&1 || { cat "$O/ab_${c}_$mode.log"; exit 1; }
    echo "$mode: $(grep -v amdgpu.ids "$O/ab_${c}_$mode.log" | cut -c1-330)"
  done
done
