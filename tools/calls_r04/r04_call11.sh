#!/bin/bash
# round 4, call 11: plugin calls beside back-to-back 1 GiB batch seals (new test) and the worker tests; c4s FETCH_SIZE at
# one key with every record 8 192 B (full blocks only) and 8 200 B (a partial block each): is the c4s fetch excess over the
# record bytes the partial blocks' narrow loads (counted at a 64-B request each) or real re-reads?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c11; mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_worker.py -x -v --timeout 300 --timeout-method thread > "$O/worker_tests.log" 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" "$O/worker_tests.log" | tail -8; [ $rc -eq 0 ] || { tail -40 "$O/worker_tests.log"; exit $rc; }
P=$R/hsig-picotls_amd/libptls_hip.so
cd /tmp || exit 1
i=0
for fl in 8192 8200 0; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$O/pmc_$i" -o run -- \
      python3 "$R/tools/time_cfg.py" --config c4s --reps 3 --keys 1 --lanes 64 --fixed-len $fl $P > "$O/pmc_$i.log" 2>&1 || { tail -5 "$O/pmc_$i.log"; exit 1; }
  echo "fixed-len $fl: $(python3 "$R/tools/counter_avg.py" "$O/pmc_$i" FETCH_SIZE 2048)"
done
