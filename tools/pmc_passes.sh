#!/bin/bash
# Collect SQ/LDS counters for the batch kernel in separate rocprofv3 passes (one --pmc set each, never
# combined with tracing domains).  usage: tools/pmc_passes.sh <outdir> <bench args...>
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
set -o pipefail
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVES"
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC"
)
i=0
for p in "${passes[@]}"; do
  timeout -k 10 240 rocprofv3 --pmc $p -T --output-format csv -d "$out/pass$i" -o run -- python3 bench.py "$@" > "$out/pass$i.log" 2>&1 || exit $?
  i=$((i+1))
done
