#!/bin/bash
# round 4, call 1: the GPU suite on the chunk-queue build, then a same-box A/B of the chunk queue (product) against the
# static grid stride (variants/libptls_hip_noqueue.so) on c2 / c3 / c4 with the per-workgroup finish spread
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c1; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so; V=$R/hsig-picotls_amd/variants/libptls_hip_noqueue.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
for c in c2 c3 c4; do
  timeout -k 10 240 python -u tools/time_cfg.py --config $c --clock $V $P $V $P > "$O/ab_$c.log" 2>&1 || { cat "$O/ab_$c.log"; exit 1; }
  cat "$O/ab_$c.log"
done
