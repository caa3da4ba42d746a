#!/bin/bash
# round-end evidence refresh (part 1): c2, c3 -- kernel stats, HBM traffic, SQ/LDS counters, full bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 1100 tools/refresh_profiles.sh r02 c2 c3
