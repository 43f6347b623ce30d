#!/bin/bash
# cross-stream interference reproducer: encoder plan (B-direct on / off in the
# encoder) replaying on a side stream while matching runs on the main stream
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
STRESS_SECONDS=25 timeout -k 10 150 python -u tools/stress_bd_concurrency.py > $O/stress_on.log 2>&1 || { tail -5 $O/stress_on.log; exit 1; }
grep RESULT $O/stress_on.log
S3_GEMM_BDIRECT_OFF=enc STRESS_SECONDS=25 timeout -k 10 200 python -u tools/stress_bd_concurrency.py > $O/stress_off.log 2>&1 || { tail -5 $O/stress_off.log; exit 1; }
grep RESULT $O/stress_off.log
