#!/bin/bash
set -o pipefail
O=gpurun_out/r06g2w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_gaussians.py tests/test_gaussian_map.py tests/test_pairs.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -15 $O/tests.log; exit $rc
