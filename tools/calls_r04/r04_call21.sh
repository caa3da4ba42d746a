#!/bin/bash
# round 4, call 21: multi-device rehearsals for the driver's N > 1 runs on the one-GPU box: the node API with device 0
# listed eight times (c2, 1 GiB, host memory bound per entry's NUMA node) and bench.py at four ranks on device 0 through
# torch.distributed.run (the launcher the driver uses), per-rank parity, host_e2e_node at N > 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c21; mkdir -p "$O"
timeout -k 10 300 python -u bench.py --node-e2e 0,0,0,0,0,0,0,0 --config c2 > "$O/node8.json" 2> "$O/node8.err" || { tail -20 "$O/node8.err"; exit 1; }
tail -1 "$O/node8.json" | cut -c1-1500
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 4 --device 0 --steps 3 --warmup 1 --records 65536 --e2e-records 16384 > "$O/ranks4.json" 2> "$O/ranks4.err" || { tail -30 "$O/ranks4.err"; exit 1; }
tail -1 "$O/ranks4.json" | cut -c1-2500
