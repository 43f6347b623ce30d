#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_end_tests.log 2>&1 || { tail -30 gpurun_out/r05_end_tests.log; exit 1; }
tail -1 gpurun_out/r05_end_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_end_smoke.log 2>&1 || { tail -20 gpurun_out/r05_end_smoke.log; exit 1; }
tail -1 gpurun_out/r05_end_smoke.log
