#!/bin/bash
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in 1000000 4000000 16000000; do
DIAG_ENC_SLEEP=$c DIAG_TRIALS=3 timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag_$c.log 2>&1 || { tail -5 $O/diag_$c.log; exit 1; }
echo "sleep $c:"; grep -E "^trial|live !=" $O/diag_$c.log | cut -c1-160
done
for c in 4000000; do
S3_GEMM_BDIRECT_OFF=enc DIAG_ENC_SLEEP=$c DIAG_TRIALS=3 timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag_off_$c.log 2>&1 || { tail -5 $O/diag_off_$c.log; exit 1; }
echo "bd off in enc, sleep $c:"; grep -E "^trial|live !=" $O/diag_off_$c.log | cut -c1-160
done
