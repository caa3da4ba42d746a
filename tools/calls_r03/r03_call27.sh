#!/bin/bash
# round 3, call 27: the committed final tree (basis plane H^128): smoke, default bench line, c4 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r03c27; mkdir -p "$O"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python bench.py > "$O/bench.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$O/bench.log"; exit 1; }
grep '"metric"' "$O/bench.log" | cut -c1-420
timeout -k 10 400 python bench.py --config c4 --no-e2e --no-plugin > "$O/bench_c4.log" 2>&1 || { echo "bench c4 rc=$?"; tail -20 "$O/bench_c4.log"; exit 1; }
grep '"metric"' "$O/bench_c4.log" | cut -c1-420
