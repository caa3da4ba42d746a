# round 6: per-call latency of several builds of the four-wave plugin worker, alternating (variants named in $VARIANTS,
# "prod" = the in-tree library), after the plugin-size and worker tests
set -o pipefail
OUT=gpurun_out/${OUT:-r06split_ab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plugin_sizes.py tests/test_gpu_worker.py > $OUT/tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in $VARIANTS; do
    if [ $v = prod ]; then lib=hsig-picotls_amd/libptls_hip.so; else lib=hsig-picotls_amd/variants/libptls_hip_$v.so; fi
    echo "== $v" >> $OUT/calls.log
    PTLS_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/plugin_calls.py 2000 >> $OUT/calls.log 2>&1 || exit 1
  done
done
