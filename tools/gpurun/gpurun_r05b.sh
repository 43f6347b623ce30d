#!/bin/bash
# round 5: GPU tests touched by the hygiene changes (pp tiles, libm-exp oracle, render flags, spin)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_net_ops.py tests/test_raster.py tests/test_slam.py tests/test_tune_db.py > gpurun_out/r05b_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05b_tests.log; exit $rc
