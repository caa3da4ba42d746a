#!/bin/bash
# round 4, call 31: round-end evidence refresh on the session-2 kernels (+ WIN_ALL windowed combination for every G, G = 4 for long key runs; DPP reductions, sparse AAD prefetch, window-table
# rows), part 1 (c2 c3): kernel trace + stats, HBM traffic, SQ / LDS counter passes, full bench lines (tools/refresh_profiles.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 tools/refresh_profiles.sh r04 c2 c3
