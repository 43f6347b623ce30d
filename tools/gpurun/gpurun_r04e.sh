#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_matching.py tests/test_slam.py -k "refine or match or decode_ahead" -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1 || { tail -40 gpurun_out/r04e_tests.log; exit 1; }
grep -E "passed|slots" gpurun_out/r04e_tests.log
timeout -k 10 300 python -u -m tools.bench_match > gpurun_out/r04e_match.log 2>&1 || { tail -20 gpurun_out/r04e_match.log; exit 1; }
cat gpurun_out/r04e_match.log
