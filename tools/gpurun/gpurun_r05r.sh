#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05r
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r05r/prof -o run -- python3 bench.py --steps 12 --warmup 4 $OFF > gpurun_out/r05r/prof.log 2>&1 || { tail -20 gpurun_out/r05r/prof.log; exit 1; }
timeout -k 10 200 python3 -m tools.rocprof_issue gpurun_out/r05r/prof/run_results.db --last-ms 60 --min-gap-us 25 > gpurun_out/r05r/issue.txt 2>&1
rc=$?; rm -rf gpurun_out/r05r/prof; tail -3 gpurun_out/r05r/issue.txt; exit $rc
