#!/bin/bash
# round 3, call 19: round-end evidence refresh for c2 c3 (kernel stats, HBM traffic, SQ/LDS passes, full bench lines) on the
# final build: tools/refresh_profiles.sh, collected afterwards with tools/collect_profiles.sh r03 c2 c3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 bash tools/refresh_profiles.sh r03 c2 c3 || { echo "refresh rc=$?"; exit 1; }
for c in c2 c3; do grep '"metric"' gpurun_out/bench_${c}_full.log | cut -c1-400; done
