set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ssao" --timeout 120 --timeout-method thread > gpurun_out/halo_test.log 2>&1 || { tail -30 gpurun_out/halo_test.log; exit 1; }
tail -2 gpurun_out/halo_test.log
for h in 0 8 16 32; do echo "== halo $h"; SOC_SSAO_HALO=$h bash tools/kt_quick.sh | grep -i ssao_k || exit 1; done
