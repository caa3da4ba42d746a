#!/bin/bash
# round 5, call 15 (rerun as the final refresh after calls 18-24 changed the generic loads): round-end evidence for c2 and c3 on the round's product (tools/refresh_profiles.sh: kernel trace +
# stats, FETCH_SIZE / WRITE_SIZE passes, SQ / LDS passes, a full bench line each with the CPU baseline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 tools/refresh_profiles.sh r05 c2 c3
