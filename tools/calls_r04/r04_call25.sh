#!/bin/bash
# round 4, call 25: WIN_ALL variant (every G >= 2 combines by one windowed multiply per lane + an XOR over the record's lanes,
# instead of the nibble-table tree and its final multiply by H): the parity file on the variant, then same-box A/B against
# the product on c3 (G = 4), c2 (G = 8) and c4's lengths at ~105 records per key (G = 16), alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04c25; mkdir -p "$O"; V=$R/hsig-picotls_amd/variants
PTLS_HIP_LIB=$V/libptls_hip_winall.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/parity.log" 2>&1
rc=$?; tail -2 "$O/parity.log"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/parity.log" | head -20; exit $rc; }
for a in "--config c3" "--config c2" "--config c4 --keys 40000"; do
  for n in prod winall prod winall; do
    timeout -k 10 200 python -u tools/time_cfg.py $a $V/libptls_hip_$n.so > "$O/ab.log" 2>&1 || { cat "$O/ab.log"; exit 1; }
    grep -v amdgpu.ids "$O/ab.log" | cut -c1-200
  done
done
