#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05blend
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_raster.py tests/test_n1.py > gpurun_out/r05blend/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05blend/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m tools.bench_raster --iters 10 > gpurun_out/r05blend/c3.log 2>&1 || { tail -5 gpurun_out/r05blend/c3.log; exit 1; }
grep '^{' gpurun_out/r05blend/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('fwd_ms','fwd_deferred_ms','deferred_equal','bwd_ms','phases_ms')})"
