#!/bin/bash
# tuner decisions of the bench's batched plans, then attention kernel variants at that composition
set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
S3_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u bench.py $Q > gpurun_out/tune_log.log 2>&1 || { tail -20 gpurun_out/tune_log.log; exit 1; }
grep 'gemm-tune' gpurun_out/tune_log.log | grep -E '^\[gemm-tune\] (6144|1536|768)x' | head -60
grep '^{' gpurun_out/tune_log.log | python -c "import json,sys; print('fps', json.loads(sys.stdin.read())['value'])"
bash tools/gpurun/gpurun_r03p.sh
