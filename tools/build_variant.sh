#!/bin/bash
# build a tuning variant of the engine: tools/build_variant.sh <threads> <pure_blocks> -> hsig-picotls_amd/variants/libptls_hip_<t>_<k>.so
set -e
cd "$(dirname "$0")/../hsig-picotls_amd"
t=$1; k=$2; out=variants/libptls_hip_${t}_${k}.so
mkdir -p variants/build_${t}_${k}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -DPTLS_HIP_WG_THREADS=$t -DPURE_BLOCKS=$k $EXTRA -I../include -Icsrc -c csrc/aesgcm_kernels.hip -o variants/build_${t}_${k}/k.o
g++ -std=c++17 -O2 -fPIC -D__HIP_PLATFORM_AMD__ -DPTLS_HIP_WG_THREADS=$t -I/opt/rocm/include -I../include -Icsrc -c csrc/engine.cpp -o variants/build_${t}_${k}/e.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out variants/build_${t}_${k}/k.o variants/build_${t}_${k}/e.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPTLS_HIP_WG_THREADS=$t -DPURE_BLOCKS=$k $EXTRA -I../include -Icsrc -c csrc/aesgcm_kernels.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A6 "ILi8ELi10ELb0ELb1" | grep -E "VGPRs:|Scratch" | sed "s/^.*remark: */$t x $k: /"
