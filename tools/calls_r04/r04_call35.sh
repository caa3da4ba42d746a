#!/bin/bash
# round 4, call 35: the session's final tree (+ the table build's opaque thread index: no scratch left in any batch
# instantiation): GPU suite (with the rebuilt test-only builds), smoke, same-box A/B against the previous product (final0)
# on c4 / c3 / c2, default bench line, plugin probe and the multi-thread plugin run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c35; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants; P=$R/hsig-picotls_amd/libptls_hip.so
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
for c in c4 c3 c2; do
  for L in $V/libptls_hip_final0.so $P $V/libptls_hip_final0.so $P; do
    timeout -k 10 200 python -u tools/time_cfg.py --config $c $L > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
timeout -k 10 400 python -u bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" || { tail "$O/bench_c2.err"; exit 1; }
python -c "import json;r=json.loads(open('$O/bench_c2.json').read().splitlines()[-1]);print('c2', r['config']['lanes_per_record'], r['seal_gibps'], r['open_gibps'], r['value'], r['roofline']['frac'], r['clock_in_run']['seal_ghz'], r['clock_in_run']['seal_finish_spread'], r['host_e2e']['seal_open_gibps'], r['cpu_baseline']['value'], r['plugin_ptlsbench']['hip_aes128gcm']['enc_us_per_call'])"
timeout -k 10 120 python -u tools/plugin_probe.py > "$O/probe.json" 2>/dev/null && cat "$O/probe.json" || exit 1
timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt.json" 2> "$O/plugin_mt.err" && cut -c1-800 "$O/plugin_mt.json" || { tail "$O/plugin_mt.err"; exit 1; }
