#!/bin/bash
# FP64 victim vs our MFMA GEMM; matching victim vs a hipBLASLt GEMM of the same shape
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { env "$@" STRESS_SECONDS=12 timeout -k 10 90 python -u tools/stress_bd_concurrency.py > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }; grep RESULT $O/s.log; }
run STRESS_SIDE=gemm25 STRESS_VICTIM=torch64
run STRESS_SIDE=torchs STRESS_VICTIM=match
run STRESS_SIDE=torchs STRESS_VICTIM=torch64
run STRESS_SIDE=torch STRESS_VICTIM=torch64
