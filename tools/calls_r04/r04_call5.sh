#!/bin/bash
# round 4, call 5: stream-ordered allocation of keysets / batches (no device-wide hipFree), worker life knobs -- the GPU
# suite, the plugin measurements at 8 and 16 mailboxes, then the default bench line (c2) with the new CPU baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c5; mkdir -p "$O"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; grep -E "passed|failed|error" "$O/gpu_tests.log" | tail -3; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/gpu_tests.log" | head -30; exit $rc; }
timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt8.json" 2> "$O/plugin_mt8.err" || { tail -20 "$O/plugin_mt8.err"; exit 1; }
cat "$O/plugin_mt8.json"; echo
PTLS_HIP_PLUGIN_WORKERS=16 timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt16.json" 2> "$O/plugin_mt16.err" || { tail -20 "$O/plugin_mt16.err"; exit 1; }
cat "$O/plugin_mt16.json"; echo
timeout -k 10 400 python -u bench.py > "$O/bench_c2.json" 2> "$O/bench_c2.err" || { tail -20 "$O/bench_c2.err"; exit 1; }
cat "$O/bench_c2.json"
