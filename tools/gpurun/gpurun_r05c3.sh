#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05c3
timeout -k 10 200 python -u -m tools.bench_raster --iters 10 > gpurun_out/r05c3/c3.log 2>&1 || { tail -5 gpurun_out/r05c3/c3.log; exit 1; }
grep '^{' gpurun_out/r05c3/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('fwd_ms','fwd_deferred_ms','deferred_equal','bwd_ms','phases_ms')})"
