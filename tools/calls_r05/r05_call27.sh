#!/bin/bash
# round 5, call 27: the sparse kernel's seal folds the stretch's last two ciphertext blocks into the first tail pair's
# skewed AES (the kernel is latency-bound per wave): GPU suite, base (variants/libptls_hip_base.so = the previous product)
# vs new alternating on c4s, and the plugin per-call latency of both (tools/plugin_probe.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c27; mkdir -p "$O"
V=$R/hsig-picotls_amd/variants; B=$V/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N $B $N --config c4s 2>&1 | grep GiB > "$O/ab.log" || exit 1
cat "$O/ab.log"
for L in $B $N $B $N; do
  PTLS_HIP_LIB=$L timeout -k 10 200 python -u tools/plugin_probe.py 2>&1 | grep '^{' || exit 1
done > "$O/plugin.log"
cut -c1-400 "$O/plugin.log"
