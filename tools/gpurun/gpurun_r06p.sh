#!/bin/bash
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
DIAG_MAIN_PRIORITY=0 DIAG_TRIALS=4 timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag_prio0.log 2>&1 || { tail -5 $O/diag_prio0.log; exit 1; }
echo "main priority 0:"; grep -E "^trial|live !=" $O/diag_prio0.log | cut -c1-200
DIAG_TRIALS=2 timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag_default.log 2>&1 || { tail -5 $O/diag_default.log; exit 1; }
echo "default:"; grep -E "^trial|live !=" $O/diag_default.log | cut -c1-200
