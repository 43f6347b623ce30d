#!/bin/bash
# round 5: cached device projection matrix: render / frontend tests, then the driver command x5
set -o pipefail
mkdir -p gpurun_out/r05proj
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_slam.py tests/test_raster.py tests/test_n1.py tests/test_host_glue.py tests/test_gaussian_map.py > gpurun_out/r05proj/tests.log 2>&1
rc=$?; tail -1 gpurun_out/r05proj/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpurun/gpurun_r05rep.sh
