#!/bin/bash
# render worker: equality tests, then headline A/B (render worker on / off) and the end-to-end leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_slam.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/slam_tests.log 2>&1 || { tail -40 gpurun_out/slam_tests.log; exit 1; }
tail -1 gpurun_out/slam_tests.log
CONFIGS=" ;--no-render-async; ;--no-render-async" bash tools/gpurun/gpurun_ab.sh || exit 1
Q="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-kprof"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/e2e_run.log 2>&1 || { tail -30 gpurun_out/e2e_run.log; exit 1; }
grep '^{' gpurun_out/e2e_run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('device', round(d['value'],1), 'e2e', round(d['end_to_end_fps'],1))"
