#!/bin/bash
# round 5: where the decoder-shape GEMM launches spend their time (debug-flag decomposition)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m tools.bench_gemm_parts \
  --shapes 1536x768x768x2,1536x2304x768x2,1536x3072x768x2,1536x768x3072x2,1536x1536x768x2,6144x4096x1024x1,6144x1024x4096x1 \
  --tiles 32,37,26,22,28,1,5,27 > gpurun_out/r05a_parts.log 2>&1
