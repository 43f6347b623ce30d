#!/bin/bash
# round 5: host wake-up A/B for the GN wait (spin budget)
set -o pipefail
mkdir -p gpurun_out/r05t
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live"
for n in 1 2 3; do
  for S in 1000 20000; do
    S3_SPIN_US=$S timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05t/one.log 2>&1 || { tail -20 gpurun_out/r05t/one.log; exit 1; }
    grep '^{' gpurun_out/r05t/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('spin_us=$S run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', c['big_gaps'])" | tee -a gpurun_out/r05t/ab.log
  done
done
