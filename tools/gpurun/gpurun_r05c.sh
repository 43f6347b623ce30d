#!/bin/bash
# round 5: GEMM op tests (new tiles, vector-epilogue rule) + deep-ring tile decomposition on the decoder shapes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_net_ops.py tests/test_raster.py > gpurun_out/r05c_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m tools.bench_gemm_parts \
  --shapes 1536x768x768x2,1536x2304x768x2,1536x3072x768x2,1536x768x3072x2,1536x1536x768x2 \
  --tiles 32,26,33,38,39 > gpurun_out/r05c_parts.log 2>&1
