#!/bin/bash
# round 5: frame-loop / backend / pairs GPU tests, then the attention + host-stall experiment
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_backend_shard.py tests/test_slam.py tests/test_pairs.py tests/test_tune_db.py tests/test_gaussians.py > gpurun_out/r05f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05f_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpurun/gpurun_r05e.sh
