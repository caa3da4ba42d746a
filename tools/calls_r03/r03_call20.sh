#!/bin/bash
# round 3, call 20: round-end evidence refresh for c4 c4s (kernel stats, HBM traffic, SQ/LDS passes, full bench lines) on the
# final build: tools/refresh_profiles.sh, collected afterwards with tools/collect_profiles.sh r03 c4 c4s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 bash tools/refresh_profiles.sh r03 c4 c4s || { echo "refresh rc=$?"; exit 1; }
for c in c4 c4s; do grep '"metric"' gpurun_out/bench_${c}_full.log | cut -c1-400; done
