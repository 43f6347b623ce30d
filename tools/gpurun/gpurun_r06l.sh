#!/bin/bash
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag.log 2>&1; echo "rc=$?"; cat $O/diag.log | grep -v amdgpu.ids | cut -c1-250
