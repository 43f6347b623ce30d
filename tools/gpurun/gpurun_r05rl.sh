#!/bin/bash
# round 5: LDS-staged refine_matches: parity tests, then the tracking-loop timing
set -o pipefail
D=gpurun_out/r05rl
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_matching.py > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m tools.bench_refine > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
grep -v amdgpu.ids $D/bench.log | tail -14
