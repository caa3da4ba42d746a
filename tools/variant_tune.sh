#!/bin/bash
# same-box comparison of tuning variants: tools/tune.py on the main library, then on every variant
# usage: tools/variant_tune.sh "<tune args>"   (each run under its own time limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args=${1:-"--configs c2,c3 --lanes 4,8 --wg 768"}
echo "== main"
timeout -k 10 200 python tools/tune.py $args || exit $?
for so in hsig-picotls_amd/variants/*.so; do
  v=$(basename $so .so); alt=$(echo $v | sed -n 's/.*_w\([0-9]*\)k.*/\1/p')
  echo "== $v"
  PTLS_HIP_LIB=$so timeout -k 10 200 python tools/tune.py ${args/--wg 768/--wg ${alt:-768}} || exit $?
done
