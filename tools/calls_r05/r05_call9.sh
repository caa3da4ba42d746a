#!/bin/bash
# round 5, call 9: FETCH_SIZE / WRITE_SIZE calibration on line-offset copies (tools/copy_calib.py), then bench.py --align 16
# on c3 (the new bench mode) once, un-profiled
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c9; mkdir -p "$O"
timeout -k 10 120 python3 tools/copy_calib.py run > "$O/calib_plain.log" 2>&1 || { tail "$O/calib_plain.log"; exit 1; }
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o run -- \
      python3 "$R/tools/copy_calib.py" run > "$O/pmc_$c.log" 2>&1 || { echo "pmc $c rc=$?"; tail "$O/pmc_$c.log"; exit 1; }
done
python3 "$R/tools/copy_calib.py" parse "$O" > "$O/copy_calib.json" && cat "$O/copy_calib.json"
cd "$R"
timeout -k 10 300 python3 -u bench.py --config c3 --align 16 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-plugin > "$O/bench_c3_align16.log" 2>&1 || { tail "$O/bench_c3_align16.log"; exit 1; }
grep '^{' "$O/bench_c3_align16.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['seal_gibps'], d['open_gibps'], d['config'])"
