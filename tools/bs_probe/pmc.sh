#!/bin/bash
# PMC passes over the bit-sliced probe (one --pmc set per run)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/bs_pmc; mkdir -p $out
export TMPDIR=/tmp
i=0
for p in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA" \
         "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES"; do
  timeout -s KILL 60 rocprofv3 --pmc $p -T --output-format csv -d $out/pass$i -o run -- "$@" > $out/pass$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $out/pass$i.log; }
  i=$((i+1))
done
for f in $(find $out -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(float); n=collections.Counter()
for r in rows:
    if 'bs_ctr' not in r.get('Kernel_Name',''): continue
    agg[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k,v in agg.items(): print(f"{k:32s} {v:16.4g}  (dispatch-rows {n[k]})")
PY
done
