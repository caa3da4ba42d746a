#!/bin/bash
# round 5, call 22: the round's final tree as the driver runs it: smoke(), then `python bench.py` with no flags (N = 1,
# configs[1], CPU baseline, host-resident and plugin timings), and the same under rocprofv3 --kernel-trace --stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c22; mkdir -p "$O"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py > "$O/bench_default.log" 2>&1 || { tail "$O/bench_default.log"; exit 1; }
grep '^{' "$O/bench_default.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['seal_gibps'], d['open_gibps'], d['roofline']['frac'], d['roofline']['measured_copy_gbs'], d['cpu_baseline']['value'], d['cpu_baseline']['full_host_extrapolation']['gibps'], d['host_e2e']['seal_open_gibps'])"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_trace.log" 2>&1 || { echo "trace rc=$?"; tail "$O/bench_trace.log"; exit 1; }
python3 "$R/tools/trace_summary.py" "$O/trace/run_kernel_trace.csv" > "$O/kernel_trace_summary.json" 2>&1; cat "$O/kernel_trace_summary.json"
