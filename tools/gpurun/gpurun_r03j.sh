#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m tools.bench_conv_parts --tiles 4,3,28,40,41,42,43,45 --B 2 > gpurun_out/conv_parts.log 2>&1 || { tail -20 gpurun_out/conv_parts.log; exit 1; }
grep conv gpurun_out/conv_parts.log
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py tests/test_gaussians.py tests/test_host_glue.py tests/test_gaussian_map.py tests/test_slam.py::test_decode_ahead_frontend_matches_sequential -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/g2w_tests.log 2>&1 || { tail -40 gpurun_out/g2w_tests.log; exit 1; }
tail -1 gpurun_out/g2w_tests.log
CONFIGS="--enc-batch 8 --enc-ahead 8;--enc-batch 8 --enc-ahead 8 --main-priority 0" bash tools/gpurun/gpurun_ab.sh && S3_GEMM_HALO=0 CONFIGS="--enc-batch 8 --enc-ahead 8" bash tools/gpurun/gpurun_ab.sh
