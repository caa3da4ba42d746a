#!/bin/bash
# plugin-call latency: product build and sparse-kernel ablations (no AES table build / no combination / no H^64 table),
# then the product build's kernel time under rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
V=hsig-picotls_amd/variants
steps=("base:120:python tools/plugin_probe.py")
for n in plugnotab nocomb noh64; do steps+=("$n:120:PTLS_HIP_LIB=$V/libptls_hip_$n.so python tools/plugin_probe.py"); done
tools/gpu_steps.sh "${steps[@]}" && \
  cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/plugprof" -o plug -- python3 "$GRAFT_REPO_ROOT/tools/plugin_probe.py" > "$GRAFT_REPO_ROOT/gpurun_out/plugprof.log" 2>&1; echo "rocprof rc=$?"
