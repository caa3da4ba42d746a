#!/bin/bash
# Copy the summaries written by tools/refresh_profiles.sh from gpurun_out/ into profiles/ (committed).
set -e
cd "$(dirname "$0")/.."
tag=${1:-r02}; shift || true
cfgs=${*:-c2 c3 c4 c4s}
for c in $cfgs; do
  cp gpurun_out/prof_${tag}_$c/trace/run_kernel_stats.csv profiles/${tag}_${c}_kernel_stats.csv
  # per-launch seal / open durations of the batch kernels, the engine self-check dispatches dropped (rocprofv3's stats
  # average them in), from the very trace the stats came from
  python3 tools/trace_summary.py gpurun_out/prof_${tag}_$c/trace/run_kernel_trace.csv > profiles/${tag}_${c}_kernel_trace_summary.json
  cp gpurun_out/prof_${tag}_$c/traffic_$c.json profiles/traffic_$c.json
  cp gpurun_out/pmc_$c/lds_$c.json profiles/lds_$c.json
  cp gpurun_out/pmc_$c/summary.txt profiles/${tag}_${c}_pmc_sq_summary.txt
  grep '"metric"' gpurun_out/bench_${c}_full.log > profiles/${tag}_bench_${c}_latest.log
  # the raw rocprofv3 CSVs the summaries above are computed from (kernel trace, HBM counter passes, SQ / LDS passes),
  # so that a reader can re-derive them: tools/trace_summary.py, tools/traffic_json.py, tools/pmc_summary.py
  raw=profiles/raw_${tag}/$c; mkdir -p $raw
  cp gpurun_out/prof_${tag}_$c/trace/run_kernel_trace.csv $raw/kernel_trace.csv
  for k in FETCH_SIZE WRITE_SIZE; do
    cp gpurun_out/prof_${tag}_$c/pmc_$k/run_counter_collection.csv $raw/pmc_$k.csv
  done
  for d in gpurun_out/pmc_$c/pass*/; do
    cp "$d"run_counter_collection.csv $raw/sq_$(basename "$d").csv
  done
done
