#!/bin/bash
# conv tail with fp32 weights in LDS: network goldens + conv parts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_net.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1 || { tail -30 gpurun_out/r04r_tests.log; exit 1; }
tail -1 gpurun_out/r04r_tests.log
timeout -k 10 300 python -u -m tools.bench_conv_parts --tiles 51,52 --B 2 > gpurun_out/r04r_conv_parts.log 2>&1 || { tail -20 gpurun_out/r04r_conv_parts.log; exit 1; }
grep conv gpurun_out/r04r_conv_parts.log
