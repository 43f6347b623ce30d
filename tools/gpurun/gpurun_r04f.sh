#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_matching.py -k "refine or match" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1 || { tail -40 gpurun_out/r04f_tests.log; exit 1; }
tail -2 gpurun_out/r04f_tests.log
timeout -k 10 300 python -u -m tools.refine_stats > gpurun_out/r04f_stats.log 2>&1 || { tail -30 gpurun_out/r04f_stats.log; exit 1; }
grep call gpurun_out/r04f_stats.log
