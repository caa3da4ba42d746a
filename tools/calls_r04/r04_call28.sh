#!/bin/bash
# round 4, call 28: 4 against 8 lanes per record for mid-size records on the WIN_ALL build (fixed 3 000 / 4 096 / 8 192 B,
# c3's record count scaled to ~5 GiB), same box, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c28; mkdir -p "$O"; P=$R/hsig-picotls_amd/libptls_hip.so
run() { timeout -k 10 200 python -u tools/time_cfg.py "$@" $P > "$O/t.log" 2>&1 || { cat "$O/t.log"; exit 1; }; echo "$* :: $(grep -v amdgpu.ids $O/t.log | cut -c20-150)"; }
for k in 1 2; do for g in 4 8; do run --config c3 --fixed-len 3000 --records 1887436 --lanes $g; done; done
for k in 1 2; do for g in 4 8; do run --config c3 --fixed-len 4096 --records 1382400 --lanes $g; done; done
for k in 1 2; do for g in 4 8; do run --config c3 --fixed-len 8192 --records 691200 --lanes $g; done; done
for k in 1 2; do for g in 4 8; do run --config c2 --lanes $g; done; done
