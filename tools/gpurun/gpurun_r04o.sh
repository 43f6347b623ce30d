#!/bin/bash
# tracker tests + headline bench (one finalize+solve launch per GN iteration)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_tracker.py tests/test_slam.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || { tail -30 gpurun_out/r04o_tests.log; exit 1; }
tail -1 gpurun_out/r04o_tests.log
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04o_one.log 2>&1 || { tail -20 gpurun_out/r04o_one.log; exit 1; }
  grep '^{' gpurun_out/r04o_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print(round(d['value'],1), round(d['ms_per_step'],3), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3))" | tee -a gpurun_out/r04o_ab.log
done
