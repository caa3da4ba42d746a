#!/bin/bash
# round 4, call 29: the planner's new lanes rule (G = 4 for long key runs, WIN_ALL build): GPU suite (the dealing case now also
# at G = 4), smoke, and the default bench line (c2 now at 4 lanes per record)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c29; mkdir -p "$O"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python -u bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" || { tail "$O/bench_c2.err"; exit 1; }
python -c "import json;r=json.loads(open('$O/bench_c2.json').read().splitlines()[-1]);print('c2', r['config']['lanes_per_record'], r['seal_gibps'], r['open_gibps'], r['value'], r['roofline']['frac'], r['clock_in_run']['seal_ghz'], r['clock_in_run']['seal_finish_spread'])"
