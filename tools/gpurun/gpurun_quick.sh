#!/bin/bash
# one GPU call: GPU tests (optionally a subset), per-launch network profile, bench without the CPU leg
set -o pipefail
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
(timeout -k 10 200 python -u -m tools.profile_net > gpurun_out/profile_net.log 2>&1) || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 1500 gpurun_out/bench.log
