#!/bin/bash
# round 4, call 33: round-end evidence refresh on the session-2 kernels (DPP reductions, sparse AAD prefetch, window-table
# rows), c4s after the spill fix: kernel trace + stats, HBM traffic, SQ / LDS counter passes, full bench lines (tools/refresh_profiles.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 tools/refresh_profiles.sh r04 c4s
