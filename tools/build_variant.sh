#!/bin/bash
# build a tuning variant of the engine with extra defines:
#   EXTRA="-DWG_ALT=768 -DPURE_BLOCKS=2" tools/build_variant.sh <name>  ->  hsig-picotls_amd/variants/libptls_hip_<name>.so
set -e
cd "$(dirname "$0")/../hsig-picotls_amd"
name=$1; out=variants/libptls_hip_${name}.so
mkdir -p variants/build_${name}
for src in aesgcm_kernels sparse_kernel batch_g1 batch_g2 batch_g4 batch_g8 batch_g16; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $EXTRA -I../include -Icsrc -c csrc/$src.hip -o variants/build_${name}/$src.o &
done
wait
g++ -std=c++17 -O2 -fPIC -D__HIP_PLATFORM_AMD__ $EXTRA -I/opt/rocm/include -I../include -Icsrc -c csrc/engine.cpp -o variants/build_${name}/e.o
[ -f build/keyschedule.o ] || make -s build/keyschedule.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out variants/build_${name}/aesgcm_kernels.o variants/build_${name}/batch_g*.o variants/build_${name}/sparse_kernel.o build/keyschedule.o variants/build_${name}/e.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
echo "built $out"
