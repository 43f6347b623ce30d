#!/bin/bash
# decode-early A/B (headline only) + the slam GPU tests
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for rep in 1 2; do
for cfg in "S3_DECODE_EARLY=1" "S3_DECODE_EARLY=0"; do
  env $cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04n_one.log 2>&1 || { tail -20 gpurun_out/r04n_one.log; exit 1; }
  grep '^{' gpurun_out/r04n_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('$cfg', round(d['value'],1), round(d['ms_per_step'],3), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), d['frame_breakdown']['decode_ahead'])" | tee -a gpurun_out/r04n_ab.log
done
done
