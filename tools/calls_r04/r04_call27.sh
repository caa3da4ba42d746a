#!/bin/bash
# round 4, call 27: GPU suite on the WIN_ALL product with the rebuilt test-only builds (alt/, mutants/); then 2 against 4
# (and 8) lanes per record on QUIC-size records (c3's 1 350 B, fixed 1 000 B and 2 000 B), same box, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c27; mkdir -p "$O"; P=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
run() { timeout -k 10 200 python -u tools/time_cfg.py "$@" $P > "$O/t.log" 2>&1 || { cat "$O/t.log"; exit 1; }; echo "$* :: $(grep -v amdgpu.ids $O/t.log | cut -c20-150)"; }
for k in 1 2; do for g in 2 4; do run --config c3 --lanes $g; done; done
for k in 1 2; do for g in 2 4; do run --config c3 --fixed-len 1000 --lanes $g; done; done
for k in 1 2; do for g in 2 4 8; do run --config c3 --fixed-len 2000 --lanes $g; done; done
