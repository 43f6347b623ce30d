set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_net_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ops.log 2>&1 || { tail -30 gpurun_out/t_ops.log; exit 1; }
tail -2 gpurun_out/t_ops.log
timeout -k 10 500 python -u -m tools.bench_gemm > gpurun_out/bench_gemm.log 2>&1; tail -15 gpurun_out/bench_gemm.log
