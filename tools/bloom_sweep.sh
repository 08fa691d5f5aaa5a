#!/bin/bash
# Bloom tuning sweep on the GPU: bench per-pass bloom times for several quad-kernel thresholds.
set -o pipefail
mkdir -p gpurun_out
for thr in 0 600000 2100000 100000000; do
  SOC_BLOOM_QUAD_MIN_PX=$thr timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bloom_$thr.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/bloom_$thr.json'))
print('thr $thr', d['value'], {k: v for k, v in d['ms_per_pass'].items() if 'Bloom' in k})"
done
