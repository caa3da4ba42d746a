#!/bin/bash
# round 4, call 15: where the sparse-key kernel's time goes now (c4s phase stamps, diag build), c4s bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c15; mkdir -p "$O"
timeout -k 10 200 python -u tools/sparse_stamps.py > "$O/stamps.json" 2> "$O/stamps.err" && cat "$O/stamps.json" || { tail "$O/stamps.err"; exit 1; }
timeout -k 10 200 python -u tools/time_cfg.py --config c4s --clock hsig-picotls_amd/libptls_hip.so > "$O/t.log" 2>&1 && grep -v amdgpu.ids "$O/t.log" | cut -c1-400
