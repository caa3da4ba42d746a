#!/bin/bash
# round 4, call 39: 512- against 768-thread workgroups for the final tree's c2 / c3 (4 lanes per record), same box, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c39; mkdir -p "$O"; P=$R/hsig-picotls_amd/libptls_hip.so
run() { timeout -k 10 200 python -u tools/time_cfg.py "$@" $P > "$O/t.log" 2>&1 || { cat "$O/t.log"; exit 1; }; echo "$* :: $(grep -v amdgpu.ids $O/t.log | cut -c20-150)"; }
for k in 1 2; do for w in 768 512; do run --config c2 --wg $w; done; done
for k in 1 2; do for w in 768 512; do run --config c3 --wg $w; done; done
