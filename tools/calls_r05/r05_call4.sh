#!/bin/bash
# round 5, call 4: the integer-multiply GHASH probe and a bench line with the flat copy bar
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c4; mkdir -p "$O"
timeout -k 10 120 tools/valu_probe/gf_intmul_probe > "$O/gf_intmul_probe.log" 2>&1 || { cat "$O/gf_intmul_probe.log"; exit 1; }
cat "$O/gf_intmul_probe.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-plugin --no-e2e > "$O/bench_c2.log" 2> "$O/bench_c2.err" || { tail "$O/bench_c2.err"; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_c2.log').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['seal_gibps'],d['open_gibps'],r['measured_copy_gbs'],r['torch_uint8_copy_gbs'],r['frac'],r['frac_of_measured_copy'],d['clock_in_run']['seal_ghz'])"
