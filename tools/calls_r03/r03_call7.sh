#!/bin/bash
# round 3, call 7: round-end evidence for c2 and c3 (rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE traffic, SQ / LDS
# counter passes, full bench lines; tools/refresh_profiles.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 bash tools/refresh_profiles.sh r03 c2 c3
