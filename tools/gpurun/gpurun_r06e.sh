#!/bin/bash
# refine: the pixel-major kernel vs the default on the tracking loop's inputs + parity tests
set -o pipefail
O=gpurun_out/r06e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_matching.py -x -q --timeout 300 --timeout-method thread -k "refine" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u -m tools.bench_refine > $O/refine.log 2>&1 || { tail -30 $O/refine.log; exit 1; }
tail -14 $O/refine.log
