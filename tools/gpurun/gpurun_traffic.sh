#!/bin/bash
# HBM traffic of the network kernels: two PMC passes (FETCH_SIZE, WRITE_SIZE) over one-frame replays
set -o pipefail
mkdir -p gpurun_out/traffic
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/traffic/f gpurun_out/traffic/w
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic/f -o run -- python3 -m tools.pmc_traffic run ${PMC_ARGS} > gpurun_out/traffic/log_f.txt 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/traffic/w -o run -- python3 -m tools.pmc_traffic run ${PMC_ARGS} > gpurun_out/traffic/log_w.txt 2>&1 || exit $?
python -m tools.pmc_traffic summarize gpurun_out/traffic/f gpurun_out/traffic/w ${PMC_ARGS} --out gpurun_out/traffic/traffic.json > gpurun_out/traffic/summary.txt 2>&1
st=$?
# keep only the summary (the per-dispatch CSVs are large)
find gpurun_out/traffic -name '*.csv' -size +2M -delete
exit $st
