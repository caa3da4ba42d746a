# round 6: the plugin worker on four waves (a long record split over two pairs): parity of the plugin-size and worker
# tests, per-call latency against an earlier build (variants/libptls_hip_$BASE.so, default r06head) alternating, worker phase stamps
set -o pipefail
OUT=gpurun_out/${OUT:-r06split}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_plugin_sizes.py tests/test_gpu_worker.py > $OUT/tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in head new; do
    if [ $v = head ]; then lib=hsig-picotls_amd/variants/libptls_hip_${BASE:-r06head}.so; else lib=hsig-picotls_amd/libptls_hip.so; fi
    echo "== $v" >> $OUT/calls.log
    PTLS_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/plugin_calls.py 2000 >> $OUT/calls.log 2>&1 || exit 1
  done
done
timeout -k 10 200 python -u tools/worker_stamps.py > $OUT/stamps.json 2> $OUT/stamps.err
