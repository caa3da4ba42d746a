#!/bin/bash
# round 5, call 2: the cleaned-up kernels (rejected variants removed, ISA unchanged but for operand order): the whole GPU
# suite (new: c4 key runs + key-switch mutant, queue-slot reuse, N>1 bench with CPU baseline), smoke, the default bench
# line, then the guard-page test last (a wrong over-read would fault the GPU there)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c2; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --ignore=tests/test_gpu_guard.py --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python -u bench.py > "$O/bench_c2.log" 2> "$O/bench_c2.err" || { tail "$O/bench_c2.err"; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_c2.log').read().strip().splitlines()[-1]);print(d['value'],d['seal_gibps'],d['open_gibps'],d['roofline']['measured_copy_gbs'],d['roofline']['torch_uint8_copy_gbs'],d['cpu_baseline']['value'],d['cpu_baseline'].get('full_host_extrapolation'))"
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py -x -v --timeout 120 --timeout-method thread > "$O/guard.log" 2>&1
rc=$?; tail -3 "$O/guard.log"; exit $rc
