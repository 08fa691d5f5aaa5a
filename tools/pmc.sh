#!/bin/bash
# PMC passes over a short bench run (each counter group in its own rocprofv3 run, kernel-trace only).
# Output: gpurun_out/pmc/<pass>/... ; summarise with tools/pmc_summary.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1"
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d gpurun_out/pmc/$name -o run -- python bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$name.log; exit $rc; fi
done
