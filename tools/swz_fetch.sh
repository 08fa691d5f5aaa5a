#!/bin/bash
# FETCH_SIZE per kernel with and without the XCD-aware tile order, plus frame time for both.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/env_sweep.sh "-" "SOC_SWZ_TAA=1 SOC_SWZ_SSAO=1 SOC_SWZ_COMP=1" || exit 1
for v in 0 1; do
  SOC_SWZ_TAA=$v SOC_SWZ_SSAO=$v SOC_SWZ_COMP=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace --output-format csv -d gpurun_out/swz$v/p1 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-frames 1 > gpurun_out/swz$v.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/swz$v.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/swz$v > gpurun_out/swz$v.json
done
python - <<'PY'
import json
a, b = (json.load(open(f"gpurun_out/swz{v}.json")) for v in (0, 1))
for k in a:
    if k.startswith("soc::") and ("ssao" in k or "taa" in k or "composition" in k):
        print(k[:40], "fetchKiB", round(a[k]["FETCH_SIZE"]), "->", round(b[k]["FETCH_SIZE"]), " tcp", round(a[k]["TCP_TOTAL_CACHE_ACCESSES_sum"]), "->", round(b[k]["TCP_TOTAL_CACHE_ACCESSES_sum"]))
PY
