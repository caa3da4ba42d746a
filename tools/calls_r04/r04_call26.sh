#!/bin/bash
# round 4, call 26: the planner's lanes-per-record thresholds re-measured on the WIN_ALL build (product): seal / open GiB/s
# of each shape at the candidate G values, same box, one pass each then the first two again
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c26; mkdir -p "$O"; P=$R/hsig-picotls_amd/libptls_hip.so
run() { timeout -k 10 200 python -u tools/time_cfg.py "$@" $P > "$O/t.log" 2>&1 || { cat "$O/t.log"; exit 1; }; echo "$* :: $(grep -v amdgpu.ids $O/t.log | cut -c20-150)"; }
for g in 2 4 8; do run --config c3 --lanes $g; done
for g in 8 16; do run --config c2 --lanes $g; done
for g in 16 32; do run --config c4 --lanes $g; done
for g in 16 32; do run --config c4 --keys 40000 --lanes $g; done
for g in 8 16; do run --config c4 --keys 32768 --lanes $g; done
for g in 8 16; do run --config c4 --keys 20000 --lanes $g; done
for g in 4 8; do run --config c3 --lanes $g; done
for g in 16 32; do run --config c4 --lanes $g; done
