#!/bin/bash
# round 4, call 6: c4's time at key switches (KS_STAMPS diagnostic build) and its length-mix / key-count decomposition on
# the shipping build; the plugin measurements with 16 mailboxes and the pool's kept memory
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c6; mkdir -p "$O"
P=$R/hsig-picotls_amd/libptls_hip.so; K=$R/hsig-picotls_amd/variants/libptls_hip_ksstamps.so
for c in c4 c2 c3; do
  timeout -k 10 120 python -u tools/keyswitch_stamps.py $K --config $c > "$O/ks_$c.log" 2>&1 || { cat "$O/ks_$c.log"; exit 1; }
  grep -v amdgpu.ids "$O/ks_$c.log"
done
timeout -k 10 120 python -u tools/keyswitch_stamps.py $K --config c4 --lanes 16 > "$O/ks_c4_g16.log" 2>&1 && grep -v amdgpu.ids "$O/ks_c4_g16.log"
for extra in "" "--fixed-len 8224" "--keys 1" "--keys 1 --fixed-len 8224" "--key-len 32 --config c2"; do
  timeout -k 10 150 python -u tools/time_cfg.py --config c4 $extra $P $P > "$O/c4_decomp.log" 2>&1 || { cat "$O/c4_decomp.log"; exit 1; }
  echo "[$extra] $(grep -v amdgpu.ids "$O/c4_decomp.log" | tail -1 | cut -c1-200)"
done
timeout -k 10 240 python -u tools/plugin_mt.py > "$O/plugin_mt16.json" 2> "$O/plugin_mt16.err" || { tail -20 "$O/plugin_mt16.err"; exit 1; }
cat "$O/plugin_mt16.json"
