#!/bin/bash
# isolate the part of k_gemm (tile 25) that corrupts concurrent kernels, and
# whether a torch-only victim is affected too
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { env "$@" STRESS_SECONDS=12 timeout -k 10 90 python -u tools/stress_bd_concurrency.py > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }; grep RESULT $O/s.log; }
run STRESS_SIDE=gemm25 STRESS_VICTIM=torch
run STRESS_SIDE=gemm25 STRESS_GEMM_DEBUG=2
run STRESS_SIDE=gemm25 STRESS_GEMM_DEBUG=4
run STRESS_SIDE=gemm25 STRESS_GEMM_DEBUG=1
run STRESS_SIDE=gemm25 STRESS_GEMM_DEBUG=8
run STRESS_SIDE=gemm25 STRESS_GEMM_DEBUG=12
