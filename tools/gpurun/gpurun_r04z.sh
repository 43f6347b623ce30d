#!/bin/bash
# k_normal_eqs wave reduce-scatter: tracker / host-glue / slam GPU tests, kernel summary of the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_tracker.py tests/test_host_glue.py tests/test_slam.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04z_tests.log 2>&1 || { tail -30 gpurun_out/r04z_tests.log; exit 1; }
tail -2 gpurun_out/r04z_tests.log
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04z_prof -o run -- python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04z_bench.log 2>&1 || { tail -20 gpurun_out/r04z_bench.log; exit 1; }
f=$(find gpurun_out/r04z_prof -name '*kernel_stats.csv' | head -1)
grep -E 'k_normal_eqs|k_finalize|k_gn_solve' "$f" | cut -c1-200
