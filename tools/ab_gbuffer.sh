#!/bin/bash
# A/B of G-buffer resolve builds: the raster GPU tests, then bench --raster with lib/libsoc_rt_orig.so and
# lib/libsoc_rt_nocap.so (variant builds linked by hand, SOC_RT_LIB_VARIANT) and the default lib with SOC_GB_TEX_PAIRS=1/0.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_raster.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_gb_tests.log 2>&1 || { tail -30 gpurun_out/ab_gb_tests.log; exit 1; }
tail -2 gpurun_out/ab_gb_tests.log
for v in orig nocap cap cap0; do
  lib=libsoc_rt.so; env=""
  [ $v = orig ] && lib=libsoc_rt_orig.so
  [ $v = nocap ] && lib=libsoc_rt_nocap.so
  [ $v = cap0 ] && env="SOC_GB_TEX_PAIRS=0"
  env SOC_RT_LIB_VARIANT=$lib $env timeout -k 10 200 python bench.py --raster --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_gb_$v.json 2> gpurun_out/ab_gb_$v.err || { tail -5 gpurun_out/ab_gb_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_gb_$v.json'));print('$v', d['value'], {k:v for k,v in d['ms_per_pass'].items() if 'GBuffer' in k or 'Depth' in k or 'Shadow' in k})"
done
