#!/bin/bash
# reduction classes picked at the batched shapes (class_batch): invariance tests, tuner log, bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_net.py tests/test_slam.py > gpurun_out/inv_tests.log 2>&1 || { tail -30 gpurun_out/inv_tests.log; exit 1; }
tail -2 gpurun_out/inv_tests.log
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-kprof"
S3_GEMM_TUNE_LOG=1 timeout -k 10 300 python -u bench.py $Q > gpurun_out/tune_log_s.log 2>&1 || { tail -20 gpurun_out/tune_log_s.log; exit 1; }
grep -E '^\[gemm-tune\] (6144|1536|768|192)x' gpurun_out/tune_log_s.log | head -80
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/b_s$i.log 2>&1 || { tail -20 gpurun_out/b_s$i.log; exit 1; }
  grep '^{' gpurun_out/b_s$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fps', d['value'], 'frac', (d.get('roofline') or {}).get('frac'))"
done
