#!/bin/bash
# one GPU call: GPU tests, smoke, default bench (all legs); logs under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -c 4000 gpurun_out/bench.log
