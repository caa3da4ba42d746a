#!/bin/bash
# round 5, call 25: an N = 2 bench line as the driver's multi-GPU runs produce it (both ranks on device 0, the one-GPU
# rehearsal), on c2's shape with a smaller shard, carrying cpu_baseline (rank 0, GPUs idle) and host_e2e_node
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c25; mkdir -p "$O"
timeout -k 10 600 python -u bench.py --gpus 2 --device 0 --records 262144 --steps 3 --warmup 1 --cpu-sample-mib 256 \
    --e2e-records 30000 --no-plugin > "$O/bench_n2.log" 2>&1 || { tail -20 "$O/bench_n2.log"; exit 1; }
grep '^{' "$O/bench_n2.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], [r['gibps'] for r in d['per_rank']], d['cpu_baseline']['value'], d['cpu_baseline']['full_host_extrapolation']['gibps'], d.get('host_e2e_node',{}).get('seal_open_gibps'))"
