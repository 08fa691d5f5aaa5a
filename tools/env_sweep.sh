#!/bin/bash
# Frame time under environment variants: tools/env_sweep.sh "ENV=a ENV2=b" "ENV=c" ...  ("-" = no env)
set -o pipefail
mkdir -p gpurun_out
i=0
for v in "$@"; do
  i=$((i+1))
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --profile-frames 10 > gpurun_out/sw_$i.json 2> gpurun_out/sw_$i.err || { echo "variant $v failed"; tail -3 gpurun_out/sw_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/sw_$i.json')); print('%-40s fps %9.1f  ms %.4f  ' % (sys.argv[1], d['value'], d['ms_per_step']) + ' '.join('%s=%.1f' % (k[:14], 1e3 * v) for k, v in d['ms_per_pass'].items()))" "${v:-default}"
done
