#!/bin/bash
# round 4, call 41: the sparse kernel's counter-mode constants by one lookup per lane (SPARSE_CTR_WAVE): GPU suite, c4s A/B
# against the previous product (before), alternating twice, plugin probe on both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c41; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants; P=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for k in 1 2; do
  for L in $V/libptls_hip_before.so $P; do
    timeout -k 10 200 python -u tools/time_cfg.py --config c4s $L > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
for L in $V/libptls_hip_before.so $P; do
  PTLS_HIP_LIB=$L timeout -k 10 120 python -u tools/plugin_probe.py > "$O/probe.json" 2>/dev/null && echo "$(basename $L) $(cut -c1-600 $O/probe.json)" || exit 1
done
