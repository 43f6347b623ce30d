set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_slam.py -m gpu -x -q --timeout 250 --timeout-method thread -k worker > gpurun_out/t_worker.log 2>&1; tail -3 gpurun_out/t_worker.log
timeout -k 10 400 python -u -m tools.bench_gemm > gpurun_out/bench_gemm.log 2>&1; tail -15 gpurun_out/bench_gemm.log
