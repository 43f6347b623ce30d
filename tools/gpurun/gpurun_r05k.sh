#!/bin/bash
# round 5: per-tile binning (raster tests both binnings, C3 A/B, rocprof of the C3 forward)
set -o pipefail
mkdir -p gpurun_out/r05k
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python -u -m tools.bench_raster --iters 10 --binning tile > gpurun_out/r05k/c3_tile.log 2>&1
rc=$?; tail -3 gpurun_out/r05k/c3_tile.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m tools.bench_raster --iters 10 --binning global > gpurun_out/r05k/c3_global.log 2>&1
rc=$?; tail -3 gpurun_out/r05k/c3_global.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_raster.py > gpurun_out/r05k/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05k/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05k/prof -o run -- python3 -m tools.bench_raster --iters 5 --no-backward > gpurun_out/r05k/prof.log 2>&1 || exit 1
head -20 gpurun_out/r05k/prof/run_kernel_stats.csv | cut -c1-160
