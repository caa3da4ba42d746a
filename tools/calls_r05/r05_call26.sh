#!/bin/bash
# round 5, call 26: the sparse kernel's per-record phase shares on c4s on the round's final code (STAMP_PHASES
# diagnostic build, tools/sparse_stamps.py), to compare with round 4's profiles/r04_c4s_phase_stamps_final.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c26; mkdir -p "$O"
timeout -k 10 300 python -u tools/sparse_stamps.py $R/hsig-picotls_amd/variants/libptls_hip_stamps.so > "$O/c4s_phases.log" 2>&1 || { tail "$O/c4s_phases.log"; exit 1; }
grep '^{' "$O/c4s_phases.log"
