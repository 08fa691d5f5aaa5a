#!/bin/bash
# Sponza-proxy mesh: GPU parity tests, then the C3 (default) / C2 / raster bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py -k "sponza_mesh" -x -v --timeout 300 --timeout-method thread > gpurun_out/mesh_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/mesh_tests.log | tail -5; [ $rc -eq 0 ] || { grep -E "^E" gpurun_out/mesh_tests.log | head -20; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench_mesh_c3.json 2> gpurun_out/bench_mesh_c3.err || { tail -5 gpurun_out/bench_mesh_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_mesh_c3.json'));print('C3', d['value'], d['config']['f_sky'], d['roofline']['frac'], d['ms_per_pass'], d['cpu_baseline'])"
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_mesh_c2.json 2> gpurun_out/bench_mesh_c2.err || { tail -5 gpurun_out/bench_mesh_c2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_mesh_c2.json'));print('C2', d['value'])"
timeout -k 10 300 python bench.py --raster --no-cpu-baseline --write-frame gpurun_out/frame_mesh_c3.png > gpurun_out/bench_mesh_raster_c3.json 2> gpurun_out/bench_mesh_raster_c3.err || { tail -5 gpurun_out/bench_mesh_raster_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_mesh_raster_c3.json'));print('C3 raster', d['value'], {k: v for k, v in d['ms_per_pass'].items() if k in ('DepthPrepass', 'SunShadowDraw', 'GBufferGeneration')})"
