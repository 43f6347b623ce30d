#!/bin/bash
# rocprofv3 kernel trace of the C3 rasterizer microbench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/rprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rprof -o run -- python3 -m tools.bench_raster --iters 5 > gpurun_out/rprof_bench.log 2>&1 || exit $?
python -m tools.rocprof_summary gpurun_out/rprof/run_results.db > gpurun_out/rprof_summary.txt 2>&1
rm -f gpurun_out/rprof/run_results.db
head -25 gpurun_out/rprof_summary.txt
