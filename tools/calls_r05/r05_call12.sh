#!/bin/bash
# round 5, call 12: the planner's small-batch rule (engine.cpp choose_lanes: raise lanes per record until every wave
# can draw two tasks): GPU suite on it, then base (variants/libptls_hip_base.so, the previous product) vs new at the
# planner's own choice, c2 / c3 at small and full sizes, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c12; mkdir -p "$O"
B=$R/hsig-picotls_amd/variants/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for spec in "c2 4096" "c2 16384" "c2 65536" "c2 0" "c3 65536" "c3 262144" "c3 0"; do
  set -- $spec
  extra=""; [ "$2" != 0 ] && extra="--records $2"
  echo "== $1 records=$2"
  timeout -k 10 200 python -u tools/time_cfg.py $B $N $B $N --config $1 $extra 2>&1 | grep GiB || exit 1
done > "$O/ab_sizes.log"
cat "$O/ab_sizes.log"
