set -o pipefail
for pr in 0 1 2; do echo "== probe $pr"; SOC_TAA_PROBE=$pr bash tools/kt_quick.sh | grep -i taa || exit 1; done
