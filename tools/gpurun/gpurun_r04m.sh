#!/bin/bash
# host cProfile of the headline timed region
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
S3_PROFILE_HOST=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04m_one.log 2> gpurun_out/r04m_host.log || { tail -20 gpurun_out/r04m_host.log; exit 1; }
grep -c . gpurun_out/r04m_host.log
