# C5 map test + frontend span profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gaussian_map.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/t_c5.log 2>&1 || { tail -40 gpurun_out/t_c5.log; exit 1; }
grep -E "c5_|passed|failed" gpurun_out/t_c5.log | tail -5
timeout -k 10 300 python -u -m tools.profile_spans --steps 40 > gpurun_out/spans.log 2>&1 || { tail -20 gpurun_out/spans.log; exit 1; }
tail -25 gpurun_out/spans.log
