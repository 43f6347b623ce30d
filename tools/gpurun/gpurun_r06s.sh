#!/bin/bash
# which aggressor corrupts concurrent matching: torch-only work, one B-direct
# GEMM tile, one LDS-staged GEMM tile of the same class
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for side in torch gemm74 gemm70 gemm25; do
STRESS_SIDE=$side STRESS_SECONDS=20 timeout -k 10 120 python -u tools/stress_bd_concurrency.py > $O/stress_$side.log 2>&1 || { tail -5 $O/stress_$side.log; exit 1; }
grep RESULT $O/stress_$side.log
done
