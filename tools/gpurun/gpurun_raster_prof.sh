#!/bin/bash
# C3 rasterizer microbench + rocprofv3 kernel trace of the forward (no backward)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python -u -m tools.bench_raster --P ${P:-4194304} --iters 10 > gpurun_out/br.log 2>&1 || { tail -20 gpurun_out/br.log; exit 1; }
tail -2 gpurun_out/br.log
rm -rf gpurun_out/rprof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/rprof -o run -- python3 -m tools.bench_raster --P ${P:-4194304} --iters 5 --no-backward > gpurun_out/br_prof.log 2>&1 || exit $?
python -m tools.rocprof_summary gpurun_out/rprof/run_results.db > gpurun_out/raster_prof.txt 2>&1
rm -f gpurun_out/rprof/run_results.db
head -30 gpurun_out/raster_prof.txt
