#!/bin/bash
# one GPU call: bench (+cpu baseline), rocprofv3 kernel stats, per-launch profile
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit $?
timeout -k 10 200 python -u -m tools.profile_net > gpurun_out/profile_net.log 2>&1
