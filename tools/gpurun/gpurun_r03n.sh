#!/bin/bash
# single-stage halo tiles (2 workgroups / CU): tests, decomposition, bench; GEMMs vs hipBLASLt at the batched shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py -k "halo" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/halo_tests.log 2>&1 || { tail -30 gpurun_out/halo_tests.log; exit 1; }
tail -1 gpurun_out/halo_tests.log
timeout -k 10 300 python -u -m tools.bench_conv_parts --tiles 3,48,50,51,52,53 --B 2 > gpurun_out/conv_parts3.log 2>&1 || { tail -20 gpurun_out/conv_parts3.log; exit 1; }
grep conv gpurun_out/conv_parts3.log
timeout -k 10 300 python -u -m tools.gemm_vs_hipblaslt > gpurun_out/gemm_vs_blt.log 2>&1 || { tail -20 gpurun_out/gemm_vs_blt.log; exit 1; }
grep 'TF' gpurun_out/gemm_vs_blt.log
CONFIGS=" ; " bash tools/gpurun/gpurun_ab.sh || exit 1
