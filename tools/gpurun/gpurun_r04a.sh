#!/bin/bash
# round 4: targeted GPU tests, the driver's exact bench command, GEMM tile ceilings
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests/test_slam.py tests/test_retrieval.py tests/test_tune_db.py tests/test_net.py tests/test_n1.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -60 gpurun_out/r04a_tests.log; exit 1; }
tail -3 gpurun_out/r04a_tests.log
T0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04a_bench.log 2> gpurun_out/r04a_bench.err || { tail -30 gpurun_out/r04a_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - T0 )) s"
tail -c 5000 gpurun_out/r04a_bench.log
timeout -k 10 300 python -u -m tools.gemm_ceiling --tiles 4,25,32,36,60,62,63,64,65,66 > gpurun_out/r04a_gemm_ceiling.log 2>&1 || { tail -20 gpurun_out/r04a_gemm_ceiling.log; exit 1; }
cat gpurun_out/r04a_gemm_ceiling.log
