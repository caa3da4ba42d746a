#!/bin/bash
# Profile evidence for one bench config, each rocprofv3 pass under its own time limit:
#   1. --kernel-trace --stats (per-kernel average duration; no counters in this pass)
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE, separate passes (HBM bytes, MI355X_MICROARCH.md)
#   4. traffic summary JSON (tools/traffic_json.py)
# usage: tools/profile_round.sh <tag> <config>    -> gpurun_out/prof_<tag>_<config>/
#        EXTRA="--align 16" adds bench arguments to every pass; PTLS_HIP_LIB selects another build of the library
tag=$1; cfg=${2:-c2}
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/prof_${tag}_${cfg}"
mkdir -p "$out"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp || exit 1
args="--config $cfg --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-plugin $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$out/trace" -o run -- \
    python3 "$root/bench.py" $args > "$out/trace.log" 2>&1 || { echo "trace pass rc=$?"; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T --output-format csv -d "$out/pmc_$c" -o run -- \
        python3 "$root/bench.py" --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-plugin $EXTRA > "$out/pmc_$c.log" 2>&1 \
        || { echo "pmc $c rc=$?"; exit 1; }
done
python3 "$root/tools/traffic_json.py" "$out" "$cfg" > "$out/traffic_$cfg.json" && cat "$out/traffic_$cfg.json"
