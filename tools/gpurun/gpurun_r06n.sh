#!/bin/bash
# decode-ahead mismatch: B-direct only in the encoder / only in the pair
# plans, and the encoder serialised against the main chain
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
n=0
for cfg in "S3_GEMM_BDIRECT_OFF=enc" "S3_GEMM_BDIRECT_OFF=pair" "DIAG_ENC_SERIAL=1"; do
n=$((n+1))
env $cfg S3_GEMM_TUNE_LOG=1 DIAG_TRIALS=3 timeout -k 10 400 python -u tools/diag_decode_ahead.py > $O/diag_$n.log 2>&1 || { echo "fail $cfg"; tail -5 $O/diag_$n.log; exit 1; }
echo "$cfg (tuned live: $(grep -c gemm-tune $O/diag_$n.log))"; grep "^trial" $O/diag_$n.log
done
