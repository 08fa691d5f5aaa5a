#!/bin/bash
# A/B environment variants on the default bench line (sky lane on). Usage: tools/ab_env.sh "K=V,K2=V2" "..." -- [bench args]
# ("" = no variables). Prints fps and per-group ms per variant.
set -o pipefail
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
i=0
for v in "${VARS[@]}"; do
  i=$((i+1))
  env ${v//,/ } timeout -k 10 200 python bench.py --steps 40 --warmup 10 --no-cpu-baseline "$@" > gpurun_out/ab_env_$i.json 2> gpurun_out/ab_env_$i.err || { echo "bench [$v] failed"; tail -5 gpurun_out/ab_env_$i.err; exit 1; }
  echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/ab_env_$i.json'));print(d['value'], d['ms_per_step'], d['ms_per_group'])")"
done
