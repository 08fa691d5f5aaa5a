set -o pipefail
bash tools/gpu.sh suite || exit 1
bash tools/gpu.sh pmc v3c "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32" -- --no-sky-lane || exit 1
bash tools/gpu.sh kt v3c --no-sky-lane || exit 1
python tools/valu_model.py --durations gpurun_out/v3c_kt gpurun_out/v3c_pmc > gpurun_out/r03c_valu_model.json && echo valu model ok
