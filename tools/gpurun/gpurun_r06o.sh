#!/bin/bash
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
DIAG_TRIALS=3 timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag.log 2>&1 || { tail -5 $O/diag.log; exit 1; }
grep -E "^trial|live !=|match [0-9]+:|prep [0-9]+:" $O/diag.log | grep -v identical | cut -c1-300
