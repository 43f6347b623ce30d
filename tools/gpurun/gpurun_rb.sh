#!/bin/bash
# raster tests (both binning modes) + C3 microbench A/B + rocprof of the forward
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_raster.py tests/test_gaussian_map.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rtests.log 2>&1 || { tail -40 gpurun_out/rtests.log; exit 1; }
tail -2 gpurun_out/rtests.log
timeout -k 10 120 python -u -m tools.bench_raster --P 4194304 --iters 10 --binning 1 > gpurun_out/br_radix.log 2>&1 || { tail -20 gpurun_out/br_radix.log; exit 1; }
tail -1 gpurun_out/br_radix.log
bash tools/gpurun/gpurun_raster_prof.sh
