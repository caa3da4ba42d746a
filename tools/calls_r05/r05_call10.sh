#!/bin/bash
# round 5, call 10: the sparse kernel's batch records on wave pairs at stride 128 (SPARSE_PAIR=1 experiment build,
# variants/libptls_hip_pair.so): parity of the lanes-64 paths on it, then c4s base vs pair (host pipelines excluded: the experiment keeps one global array of pair slots, which concurrent launches on the pipeline's streams share)
# alternating, then LDS counters and HBM traffic of the pair build's c4s
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r05c10; mkdir -p "$O"
B=$R/hsig-picotls_amd/libptls_hip.so; P=$R/hsig-picotls_amd/variants/libptls_hip_pair.so
PTLS_HIP_LIB=$P timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plugin_sizes.py -m gpu -x -q \
    -k "(64 or c4_mixed or plugin) and not pipeline" --timeout 120 --timeout-method thread > "$O/pair_tests.log" 2>&1
rc=$?; tail -2 "$O/pair_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/pair_tests.log" | head -20; exit $rc; }
timeout -k 10 300 python -u tools/time_cfg.py $B $P $B $P --config c4s > "$O/ab_c4s.log" 2>&1 || { tail "$O/ab_c4s.log"; exit 1; }
grep GiB "$O/ab_c4s.log"
export PTLS_HIP_LIB=$P
tools/pmc_passes.sh "$O/pmc_pair" --config c4s --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-plugin || { echo "pmc rc=$?"; exit 1; }
python3 tools/pmc_summary.py "$O/pmc_pair" --json "$O/lds_c4s_pair.json" > "$O/pmc_pair_summary.txt" && head -30 "$O/pmc_pair_summary.txt"
cd /tmp
T=$O/traffic; mkdir -p "$T"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c -T --output-format csv -d "$T/pmc_$c" -o run -- \
      python3 "$R/bench.py" --config c4s --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-plugin > "$T/pmc_$c.log" 2>&1 \
      || { echo "pmc $c rc=$?"; tail "$T/pmc_$c.log"; exit 1; }
done
cp "$T/pmc_FETCH_SIZE.log" "$T/trace.log"
python3 "$R/tools/traffic_json.py" "$T" c4s > "$O/traffic_c4s_pair.json" 2> "$O/traffic.err"; cat "$O/traffic_c4s_pair.json" || tail "$O/traffic.err"
