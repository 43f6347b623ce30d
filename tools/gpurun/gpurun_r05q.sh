#!/bin/bash
# round 5: headline A/B of plan branches (0 / dec / 1)
set -o pipefail
mkdir -p gpurun_out/r05q
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live"
for n in 1 2; do
  for B in 0 dec 1; do
    S3_PLAN_BRANCHES=$B timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05q/one.log 2>&1 || { tail -20 gpurun_out/r05q/one.log; exit 1; }
    grep '^{' gpurun_out/r05q/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('branches=$B run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3), 'gaps', c['big_gaps'])" | tee -a gpurun_out/r05q/ab.log
  done
done
