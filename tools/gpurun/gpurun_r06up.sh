#!/bin/bash
# upsample output pixels per thread: 2 (default) vs 4 (S3_UPSAMPLE_PX=4); the 1 vs 2 run used the same script with "for v in 1 2 1 2"
set -o pipefail
O=gpurun_out/r06up4
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_net_ops.py -x -q --timeout 300 --timeout-method thread -m gpu -k "upsample" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 2 4 2 4; do
  S3_UPSAMPLE_PX=$v timeout -k 10 120 python3 -m tools.bench_upsample > $O/px$v.log 2>&1 || { tail -5 $O/px$v.log; exit 1; }
  echo "px $v: $(grep '^{' $O/px$v.log)"
done
