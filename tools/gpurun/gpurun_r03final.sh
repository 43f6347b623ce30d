#!/bin/bash
# final round artifacts: GPU tests, smoke, full bench, rocprofv3 kernel trace of the frame loop,
# PMC traffic of the network at the bench's frame composition (encoder batch 8, Bp=2 pairs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
  tail -2 gpurun_out/tests.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
timeout -k 10 700 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 1500 gpurun_out/bench.log
STEPS=24 WIN_MS=60 GAPS=20 bash tools/gpurun/gpurun_prof.sh || exit 1
PMC_ARGS="--kb 8 --bp 2" bash tools/gpurun/gpurun_traffic.sh || exit 1
head -40 gpurun_out/traffic/summary.txt


timeout -k 10 300 python -u -m tools.bench_conv_parts --tiles 3,4,48,51,52,53 --B 2 > gpurun_out/conv_parts.log 2>&1 || { tail -20 gpurun_out/conv_parts.log; exit 1; }
grep conv gpurun_out/conv_parts.log
