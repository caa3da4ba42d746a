#!/bin/bash
# round 5, call 16: round-end evidence for c4 and c4s (as call 15)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 tools/refresh_profiles.sh r05 c4 c4s
