#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gaussians.py tests/test_host_glue.py tests/test_gaussian_map.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g2w_tests.log 2>&1
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 gpurun_out/g2w_tests.log; exit 1; }
grep -E "^(FAILED|E  )|passed|failed" gpurun_out/g2w_tests.log | head -20
bash tools/gpurun/gpurun_da.sh
