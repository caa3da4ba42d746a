#!/bin/bash
# build a tuning / ablation variant of the engine with extra defines:
#   EXTRA="-DKS_STAMPS=1" tools/build_variant.sh <name>  ->  hsig-picotls_amd/variants/libptls_hip_<name>.so
# SRCS (optional) = the kernel sources that get EXTRA (default: all); the others reuse the product build's objects.
set -e
cd "$(dirname "$0")/../hsig-picotls_amd"
make -s -j8 "$PWD/libptls_hip.so" >/dev/null  # the rule's target is the absolute path
name=$1; out=variants/libptls_hip_${name}.so
ALL="aesgcm_kernels sparse_kernel batch_g1 batch_g2 batch_g4 batch_g8 batch_g16 batch_g32"
SRCS=${SRCS:-$ALL}
mkdir -p variants/build_${name}
objs=""
for src in $ALL; do
  if [[ " $SRCS " == *" $src "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $EXTRA -I../include -Icsrc -c csrc/$src.hip -o variants/build_${name}/$src.o &
    objs="$objs variants/build_${name}/$src.o"
  else
    objs="$objs build/$src.o"
  fi
done
wait
# the host units (csrc/host.h lists them) with EXTRA as well: some switches are read by both sides
for u in engine keyset planner batch tls13 pipeline node plugin_worker plugin; do
  g++ -std=c++17 -O2 -fPIC -D__HIP_PLATFORM_AMD__ $EXTRA -I/opt/rocm/include -I../include -Icsrc -c csrc/$u.cpp -o variants/build_${name}/h_$u.o &
  objs="$objs variants/build_${name}/h_$u.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out $objs build/keyschedule.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
echo "built $out"
