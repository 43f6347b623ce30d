#!/bin/bash
# 8-wave dense tiles: op tests, GEMMs vs hipBLASLt, network parity, headline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ops_tests.log 2>&1 || { tail -30 gpurun_out/ops_tests.log; exit 1; }
tail -1 gpurun_out/ops_tests.log
timeout -k 10 300 python -u -m tools.gemm_vs_hipblaslt > gpurun_out/gemm_vs_blt2.log 2>&1 || { tail -20 gpurun_out/gemm_vs_blt2.log; exit 1; }
grep 'TF' gpurun_out/gemm_vs_blt2.log
timeout -k 10 600 python -u -m pytest tests/test_net.py tests/test_n1.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/net_tests.log 2>&1 || { tail -30 gpurun_out/net_tests.log; exit 1; }
tail -1 gpurun_out/net_tests.log
CONFIGS=" ; " bash tools/gpurun/gpurun_ab.sh || exit 1
