#!/bin/bash
# round 4, call 30: lanes per record on the new planner: c2 at 2 / 4, c4's lengths at ~210 and ~420 records per key at 4 / 8,
# c4's lengths on one key at 4 / 8; same box, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c30; mkdir -p "$O"; P=$R/hsig-picotls_amd/libptls_hip.so
run() { timeout -k 10 200 python -u tools/time_cfg.py "$@" $P > "$O/t.log" 2>&1 || { cat "$O/t.log"; exit 1; }; echo "$* :: $(grep -v amdgpu.ids $O/t.log | cut -c20-150)"; }
for k in 1 2; do for g in 2 4; do run --config c2 --lanes $g; done; done
for k in 1 2; do for g in 4 8; do run --config c4 --keys 20000 --lanes $g; done; done
for k in 1 2; do for g in 4 8; do run --config c4 --keys 10000 --lanes $g; done; done
for k in 1 2; do for g in 4 8; do run --config c4 --keys 1 --lanes $g; done; done
