set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_net_ops.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tiles or register" > gpurun_out/t_ops.log 2>&1 || { tail -30 gpurun_out/t_ops.log; exit 1; }
tail -2 gpurun_out/t_ops.log
timeout -k 10 300 python -u -m tools.bench_gemm_parts --small --tiles 1,10,6,20,21,22,23,24,25 > gpurun_out/gemm_parts_small.log 2>&1; cat gpurun_out/gemm_parts_small.log | grep -v amdgpu.ids
