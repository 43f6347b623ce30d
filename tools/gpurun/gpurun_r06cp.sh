#!/bin/bash
set -o pipefail
O=gpurun_out/r06cp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u tools/diag_copies.py > $O/copies.log 2>&1; rc=$?; grep -v amdgpu.ids $O/copies.log | tail -62; exit $rc
