#!/bin/bash
# round 5: the full GPU test suite on the current tree
set -o pipefail
mkdir -p gpurun_out/r05full
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r05full/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r05full/tests.log; exit $rc
