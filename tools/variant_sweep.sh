#!/bin/bash
# bench every built variant on c2 and c3; one JSON summary line per (variant, config)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in hsig-picotls_amd/variants/*.so; do
  for cfg in ${CFGS:-c2 c3 c4}; do
    r=$(PTLS_HIP_LIB=$so timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --no-e2e 2>/dev/null) || { echo "$so $cfg FAILED rc=$?"; exit 1; }
    echo "$(basename $so) $cfg $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["seal_gibps"], d["open_gibps"], d["parity"])')"
  done
done
