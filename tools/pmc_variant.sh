#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcv; mkdir -p $OUT
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INSTS_FLAT SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/p$i -o run -- python tools/kernel_variants.py bloom4 --run-only --modes 0 > $OUT/p$i.log 2>&1 || exit 1
done
python tools/pmc_summary.py $OUT > $OUT/summary.json
