#!/bin/bash
# round 5, call 6/7: the line-aligned stretch start (call 6) / the deferred spill stores (call 7, batch_kernel.h): GPU suite on it, then c3 at 16-byte packing and at
# 128-byte alignment, base (variants/libptls_hip_base.so, the previous product) vs new, alternating; c2 / c4 guard rows;
# then HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of c3 at 16-byte packing on the new build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c7; mkdir -p "$O"
B=$R/hsig-picotls_amd/variants/libptls_hip_base.so; N=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
for a in 16 128; do
  PTLS_BENCH_ALIGN=$a timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config c3 > "$O/ab_c3_align$a.log" 2>&1 || { tail "$O/ab_c3_align$a.log"; exit 1; }
  echo "align $a"; grep GiB "$O/ab_c3_align$a.log"
done
timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config c2 > "$O/ab_c2.log" 2>&1 || { tail "$O/ab_c2.log"; exit 1; }
grep GiB "$O/ab_c2.log"
timeout -k 10 300 python -u tools/time_cfg.py $B $N $B $N --config c4 > "$O/ab_c4.log" 2>&1 || { tail "$O/ab_c4.log"; exit 1; }
grep GiB "$O/ab_c4.log"
cd /tmp
T=$O/t16; mkdir -p "$T"
for c in FETCH_SIZE WRITE_SIZE; do
  PTLS_BENCH_ALIGN=16 timeout -k 10 120 rocprofv3 --pmc $c -T --output-format csv -d "$T/pmc_$c" -o run -- \
      python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-plugin > "$T/pmc_$c.log" 2>&1 \
      || { echo "pmc $c rc=$?"; tail "$T/pmc_$c.log"; exit 1; }
done
cp "$T/pmc_FETCH_SIZE.log" "$T/trace.log"
python3 "$R/tools/traffic_json.py" "$T" c3 > "$O/traffic_c3_align16.json" 2> "$O/traffic.err"; cat "$O/traffic_c3_align16.json" || tail "$O/traffic.err"
