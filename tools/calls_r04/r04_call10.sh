#!/bin/bash
# round 4, call 10: the sparse kernel's H^64 basis from four vectors per record (SPARSE_DERIVE=2) and its record deals
# (SPARSE_QUEUE 0 static / 2 snake / 3 snake + queue tail of 1/4 or 1/8): GPU suite, c4s A/B against the round's static
# stride + one-load basis (spstatic), FETCH_SIZE per c4s launch for spstatic, the product and one shared key; plugin_mt
# with the worker stream at the greatest priority (its own hardware queue); the product has the single-block stretch step
# (SPARSE_PURE1), pure1off the same tree without it (static0 / snake / tail8 variants are built without it too)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c10; mkdir -p "$O"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -2 "$O/gpu_tests.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/gpu_tests.log" | head -20; exit $rc; }
V=$R/hsig-picotls_amd/variants; D=$V/libptls_hip_spstatic.so; P=$R/hsig-picotls_amd/libptls_hip.so
for L in $D $V/libptls_hip_static0.so $V/libptls_hip_snake.so $V/libptls_hip_tail8.so $V/libptls_hip_pure1off.so $P $D $V/libptls_hip_static0.so $V/libptls_hip_snake.so $V/libptls_hip_tail8.so $V/libptls_hip_pure1off.so $P; do
  timeout -k 10 150 python -u tools/time_cfg.py --config c4s --clock $L > "$O/ab_c4s.log" 2>&1 || { cat "$O/ab_c4s.log"; exit 1; }
  grep -v amdgpu.ids "$O/ab_c4s.log" | cut -c1-330
done
cd /tmp || exit 1
i=0
for spec in "$D" "$P" "$P --keys 1 --lanes 64"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$O/pmc_$i" -o run -- \
      python3 "$R/tools/time_cfg.py" --config c4s --reps 3 $spec > "$O/pmc_$i.log" 2>&1 || { tail -5 "$O/pmc_$i.log"; exit 1; }
  echo "$spec: $(python3 "$R/tools/counter_avg.py" "$O/pmc_$i" FETCH_SIZE 2048)"
done
cd "$R" || exit 1
timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt.json" 2> "$O/plugin_mt.err" && cat "$O/plugin_mt.json" || { tail "$O/plugin_mt.err"; exit 1; }
