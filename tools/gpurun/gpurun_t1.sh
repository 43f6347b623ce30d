#!/bin/bash
# raster GPU tests + render glue profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_raster.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_r.log 2>&1
tail -12 gpurun_out/t_r.log
timeout -k 10 200 python -u -m tools.profile_render
timeout -k 10 200 python -u -m tools.bench_raster > gpurun_out/bench_raster.log 2>&1; tail -15 gpurun_out/bench_raster.log
