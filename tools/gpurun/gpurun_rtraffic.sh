#!/bin/bash
# C3 rasterizer: kernel summary of forward + backward, and HBM traffic (two PMC passes)
set -o pipefail
mkdir -p gpurun_out/rtraffic
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/rprof2 gpurun_out/rtraffic/f gpurun_out/rtraffic/w
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/rprof2 -o run -- python3 -m tools.bench_raster --P 4194304 --iters 5 > gpurun_out/br_fb.log 2>&1 || exit $?
python -m tools.rocprof_summary gpurun_out/rprof2/run_results.db > gpurun_out/raster_fb_prof.txt 2>&1
rm -f gpurun_out/rprof2/run_results.db
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/rtraffic/f -o run -- python3 -m tools.pmc_traffic run --workload raster > gpurun_out/rtraffic/log_f.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/rtraffic/w -o run -- python3 -m tools.pmc_traffic run --workload raster > gpurun_out/rtraffic/log_w.txt 2>&1 || exit $?
python -m tools.pmc_traffic summarize gpurun_out/rtraffic/f gpurun_out/rtraffic/w --workload raster --out gpurun_out/rtraffic/traffic.json > gpurun_out/rtraffic/summary.txt 2>&1
st=$?
find gpurun_out/rtraffic -name '*.csv' -size +2M -delete
head -30 gpurun_out/raster_fb_prof.txt
head -60 gpurun_out/rtraffic/summary.txt
exit $st
