#!/bin/bash
# round 4, call 9: the shipping tree (scalar-key worker by default, ECB through the worker): GPU suite, plugin probe +
# concurrency, default bench line, c3 / c4 / c4s bench lines; c4s with the sparse kernel's record queue against its static stride
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c9; mkdir -p "$O"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 120 python -u tools/plugin_probe.py > "$O/probe.json" 2>/dev/null && cat "$O/probe.json" || exit 1
timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt.json" 2> "$O/plugin_mt.err" && cat "$O/plugin_mt.json" || { tail "$O/plugin_mt.err"; exit 1; }
echo
timeout -k 10 400 python -u bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" && cat "$O/bench_c2.json" || { tail "$O/bench_c2.err"; exit 1; }
for c in c3 c4 c4s; do
  timeout -k 10 400 python -u bench.py --config $c --no-plugin > "$O/bench_$c.json" 2> "$O/bench_$c.err" || { tail "$O/bench_$c.err"; exit 1; }
  python -c "import json;r=json.loads(open('$O/bench_$c.json').read().splitlines()[-1]);print('$c', r['seal_gibps'], r['open_gibps'], r['value'], r['roofline']['frac'], r['clock_in_run']['seal_ghz'], r['clock_in_run']['seal_finish_spread'], r.get('host_e2e',{}).get('seal_open_gibps'), r['cpu_baseline']['value'], r['cpu_baseline'].get('engine'))"
done
S=$R/hsig-picotls_amd/variants/libptls_hip_spstatic.so; P=$R/hsig-picotls_amd/libptls_hip.so
for L in $S $P $S $P; do
  timeout -k 10 150 python -u tools/time_cfg.py --config c4s --clock $L > "$O/ab_c4s.log" 2>&1 || { cat "$O/ab_c4s.log"; exit 1; }
  grep -v amdgpu.ids "$O/ab_c4s.log" | cut -c1-330
done
