#!/bin/bash
# round 4, call 36: c4s phase stamps on the final sparse kernel (AAD prefetch, window rows, spill fix; diag build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c36; mkdir -p "$O"
timeout -k 10 200 python -u tools/sparse_stamps.py > "$O/stamps.json" 2> "$O/stamps.err" && cat "$O/stamps.json" || { tail "$O/stamps.err"; exit 1; }
timeout -k 10 200 python -u tools/time_cfg.py --config c4s --clock hsig-picotls_amd/libptls_hip.so > "$O/t.log" 2>&1 && grep -v amdgpu.ids "$O/t.log" | cut -c1-400
