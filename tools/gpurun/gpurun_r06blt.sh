#!/bin/bash
set -o pipefail
O=gpurun_out/r06blt
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m tools.gemm_vs_hipblaslt > $O/blt.log 2>&1; rc=$?; grep -v amdgpu.ids $O/blt.log; exit $rc
