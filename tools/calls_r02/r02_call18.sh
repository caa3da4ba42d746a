#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for mib in 64 128 256 512 2048; do
  for c in c2 c3 c4; do
    PTLS_HIP_MAPPED_SLICE_MIB=$mib timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-plugin --steps 1 --warmup 1 > gpurun_out/ms_${mib}_$c.log 2>&1 || exit 1
    echo "slice $mib MiB $c: $(grep -o '"mapped": {[^}]*}' gpurun_out/ms_${mib}_$c.log)"
  done
done
