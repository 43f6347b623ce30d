#!/bin/bash
# B-direct GEMM experiment: variants vs the tuner's tiles on the dense shapes
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 500 python -u -m tools.bench_gemm_bd > $O/bd.log 2>&1 || { tail -30 $O/bd.log; exit 1; }
cat $O/bd.log
