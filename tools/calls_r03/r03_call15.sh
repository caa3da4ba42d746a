#!/bin/bash
# round 3, call 15: record alignment A/B (16 / 128 bytes, PTLS_BENCH_ALIGN) on c2, c4, c4s seal/open, alternating x2, then the
# multi-rank bench test and one default bench line (128-byte layout)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c15; mkdir -p "$O"
L=$R/hsig-picotls_amd/libptls_hip.so
for rep in 1 2; do
  for A in 16 128; do
    for C in c2 c4 c4s; do
      echo "align=$A $C" >> "$O/align.log"
      PTLS_BENCH_ALIGN=$A timeout -k 10 200 python tools/time_cfg.py $L --config $C --reps 7 >> "$O/align.log" 2>&1 || { echo "time_cfg rc=$?"; tail "$O/align.log"; exit 1; }
    done
  done
done
grep -v amdgpu.ids "$O/align.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -q --timeout 300 --timeout-method thread > "$O/bench_test.log" 2>&1 \
  || { echo "bench test rc=$?"; tail -30 "$O/bench_test.log"; exit 1; }
tail -1 "$O/bench_test.log"
timeout -k 10 400 python bench.py > "$O/bench_c2.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench_c2.log"; exit 1; }
tail -1 "$O/bench_c2.log" | cut -c1-900
