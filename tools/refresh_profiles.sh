#!/bin/bash
# Round-end evidence refresh: rocprofv3 kernel stats + HBM traffic (tools/profile_round.sh), SQ/LDS counter
# passes (tools/pmc_passes.sh), and full bench lines, for c2, c3 and c4.  Outputs under gpurun_out/;
# copy the summaries into profiles/ afterwards (tools/collect_profiles.sh).
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
tag=${1:-r01}
for c in c2 c3 c4; do
  tools/profile_round.sh "$tag" $c > /dev/null
  tools/pmc_passes.sh gpurun_out/pmc_$c --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e
  python3 tools/pmc_summary.py gpurun_out/pmc_$c --json gpurun_out/pmc_$c/lds_$c.json > gpurun_out/pmc_$c/summary.txt
  # bench.py reads the LDS occupancy and traffic from profiles/: give it this run's (on the box's copy)
  cp gpurun_out/pmc_$c/lds_$c.json profiles/lds_$c.json
  cp gpurun_out/prof_${tag}_$c/traffic_$c.json profiles/traffic_$c.json
done
timeout -k 10 300 python bench.py > gpurun_out/bench_c2_full.log 2>&1
timeout -k 10 300 python bench.py --config c3 > gpurun_out/bench_c3_full.log 2>&1
timeout -k 10 300 python bench.py --config c4 > gpurun_out/bench_c4_full.log 2>&1
echo done
