#!/bin/bash
# raster + map tests, C3 microbench, rocprof of the forward
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_raster.py tests/test_gaussian_map.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rtests.log 2>&1 || { tail -40 gpurun_out/rtests.log; exit 1; }
tail -2 gpurun_out/rtests.log
bash tools/gpurun/gpurun_raster_prof.sh
