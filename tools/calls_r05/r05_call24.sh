#!/bin/bash
# round 5, call 24: the sparse kernel's batch records with the batch kernel's tail loads (generic data blocks as one
# end-anchored 16-byte load) and a branch-free AAD prefetch: GPU suite, base (variants/libptls_hip_base.so = the previous
# product) vs new alternating on c4s (latency-bound per wave: per-wave latency should show here), then c4s at 1-byte packing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c24; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; B=$V/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N $B $N --config c4s 2>&1 | grep GiB > "$O/ab.log" || exit 1
echo "c4s align 1" >> "$O/ab.log"
PTLS_BENCH_ALIGN=1 timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config c4s 2>&1 | grep GiB >> "$O/ab.log" || exit 1
cat "$O/ab.log"
