#!/bin/bash
# round 5: frame-loop / backend / pairs GPU tests after the aux-stream world records and the sharded backend
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_slam.py tests/test_backend_shard.py tests/test_pairs.py tests/test_tune_db.py tests/test_gaussians.py > gpurun_out/r05d_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r05d_tests.log; exit $rc
