#!/bin/bash
# round 3, call 22: c4s evidence refresh on the final sparse kernel (tools/refresh_profiles.sh r03 c4s)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 bash tools/refresh_profiles.sh r03 c4s || { echo "refresh rc=$?"; exit 1; }
grep '"metric"' gpurun_out/bench_c4s_full.log | cut -c1-600
