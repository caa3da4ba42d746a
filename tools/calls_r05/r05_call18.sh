#!/bin/bash
# round 5, call 18: partial blocks with independent loads (batch_kernel.h load_partial_aligned / load_bytes: one memory
# latency instead of one per byte) and dword / 16-bit / 8-bit partial stores: GPU suite, then base (variants/
# libptls_hip_base.so, the previous product) vs new alternating on c3, c4, c4s, c2, and c3 at 1-byte packing (unaligned path)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c18; mkdir -p "$O"
B=$R/hsig-picotls_amd/variants/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for c in c3 c4 c4s c2; do
  timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config $c 2>&1 | grep GiB || exit 1
done > "$O/ab.log"
PTLS_BENCH_ALIGN=1 timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config c3 2>&1 | grep GiB > "$O/ab_c3_align1.log" || exit 1
cat "$O/ab.log"; echo "c3 align 1"; cat "$O/ab_c3_align1.log"
