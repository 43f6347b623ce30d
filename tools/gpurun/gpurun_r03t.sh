#!/bin/bash
# blend pixels per thread: raster parity tests at the default (2), C3 forward A/B over S3_BLEND_PX
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_raster.py tests/test_gaussian_map.py tests/test_n1.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_raster.log 2>&1 || { tail -40 gpurun_out/t_raster.log; exit 1; }
tail -2 gpurun_out/t_raster.log
for px in 1 2 4 1 2 4; do
  S3_BLEND_PX=$px timeout -k 10 120 python -u -m tools.bench_raster --iters 20 --no-backward > gpurun_out/blend_px$px.log 2>&1 || { tail -20 gpurun_out/blend_px$px.log; exit 1; }
  grep '^{' gpurun_out/blend_px$px.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('px $px fwd_ms %.3f' % d['fwd_ms'], {k: round(v, 3) for k, v in d['phases_ms'].items()})"
done
