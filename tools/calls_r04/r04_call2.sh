#!/bin/bash
# round 4, call 2: guided chunk sizes at the end of long key runs (engine.cpp guided_tail) on the chunk-queue build:
# parity (dealing case, sweep, config samples), then a same-box A/B: static stride / queue / queue + guided tail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c2; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so; V=$R/hsig-picotls_amd/variants/libptls_hip_noqueue.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_dealing.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c2 c3 c4; do
  for mode in static queue guided; do
    case $mode in static) L=$V; G=1;; queue) L=$P; G=0;; guided) L=$P; G=1;; esac
    PTLS_HIP_GUIDED=$G timeout -k 10 120 python -u tools/time_cfg.py --config $c --clock $L > "$O/ab_${c}_$mode.log" 2>&1 || { cat "$O/ab_${c}_$mode.log"; exit 1; }
    echo "$mode: $(grep -v amdgpu.ids "$O/ab_${c}_$mode.log" | cut -c1-330)"
  done
done
