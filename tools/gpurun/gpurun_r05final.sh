#!/bin/bash
# round 5 artifacts. PART=tests: GPU tests + smoke.  PART=bench: the driver's
# bench command, rocprofv3 kernel trace of the headline frame loop, PMC
# traffic of the network at the bench's frame composition.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ "$PART" = "tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05_tests.log 2>&1 || { tail -30 gpurun_out/r05_tests.log; exit 1; }
  tail -2 gpurun_out/r05_tests.log
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.log 2>&1 || { tail -20 gpurun_out/r05_smoke.log; exit 1; }
  tail -1 gpurun_out/r05_smoke.log
  exit 0
fi
s0=$(date +%s)
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench.log 2> gpurun_out/r05_bench.err || { tail -20 gpurun_out/r05_bench.err; exit 1; }
echo "driver bench wall $(( $(date +%s) - s0 )) s"
tail -c 600 gpurun_out/r05_bench.log
STEPS=40 WIN_MS=150 GAPS=20 BENCH_ARGS="--no-live" bash tools/gpurun/gpurun_prof.sh || exit 1
head -8 gpurun_out/timeline.txt
PMC_ARGS="--kb 8 --bp 2" bash tools/gpurun/gpurun_traffic.sh || exit 1
head -30 gpurun_out/traffic/summary.txt
