#!/bin/bash
# round 4, call 37: round-end evidence refresh on the final round-4 tree (all session-2 changes; DPP reductions, sparse AAD prefetch, window-table
# rows), part 1 (c2 c3): kernel trace + stats, HBM traffic, SQ / LDS counter passes, full bench lines (tools/refresh_profiles.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 tools/refresh_profiles.sh r04 c2 c3
