#!/bin/bash
# round 4: targeted GPU tests, the driver's exact bench command, GEMM tile ceilings
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m tools.gemm_ceiling --tiles 4,25,32,36,60,62,63,64,65,66 > gpurun_out/r04a_gemm_ceiling.log 2>&1 || { tail -20 gpurun_out/r04a_gemm_ceiling.log; exit 1; }
cat gpurun_out/r04a_gemm_ceiling.log
timeout -k 10 600 python -u -m pytest tests/test_retrieval.py tests/test_slam.py tests/test_tune_db.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -40 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
/usr/bin/time -v timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench.log 2> gpurun_out/r04a_bench.err || { tail -30 gpurun_out/r04a_bench.err; exit 1; }
tail -c 3000 gpurun_out/r04a_bench.log
grep -E "Elapsed|Maximum resident" gpurun_out/r04a_bench.err
