#!/bin/bash
# bisect the decode-ahead mismatch over the frontend's side work
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
n=0
for skip in "world" "render" "world,render" ""; do
n=$((n+1))
S3_DIAG_SKIP=$skip DIAG_TRIALS=3 timeout -k 10 200 python -u tools/diag_decode_ahead.py > $O/diag_$n.log 2>&1 || { echo "fail $skip"; tail -5 $O/diag_$n.log; exit 1; }
echo "skip=[$skip]"; grep "^trial" $O/diag_$n.log
done
