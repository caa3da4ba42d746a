#!/bin/bash
# Round-end evidence refresh for the given configs (default c2 c3 c4 c4s): rocprofv3 kernel stats + HBM traffic
# (tools/profile_round.sh), SQ/LDS counter passes (tools/pmc_passes.sh), and full bench lines.  Outputs under
# gpurun_out/; copy the summaries into profiles/ afterwards (tools/collect_profiles.sh <tag> <configs>).
set -e
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
tag=${1:-r02}; shift || true
cfgs=${*:-c2 c3 c4 c4s}
for c in $cfgs; do
  echo "=== $c profile"
  tools/profile_round.sh "$tag" $c > /dev/null
  echo "=== $c pmc"
  tools/pmc_passes.sh gpurun_out/pmc_$c --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-plugin
  python3 tools/pmc_summary.py gpurun_out/pmc_$c --json gpurun_out/pmc_$c/lds_$c.json > gpurun_out/pmc_$c/summary.txt
  # bench.py reads the LDS occupancy and traffic from profiles/: give it this run's (on the box's copy)
  cp gpurun_out/pmc_$c/lds_$c.json profiles/lds_$c.json
  cp gpurun_out/prof_${tag}_$c/traffic_$c.json profiles/traffic_$c.json
  echo "=== $c bench"
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_${c}_full.log 2>&1
done
echo done
