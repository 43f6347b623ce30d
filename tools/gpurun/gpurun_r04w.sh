#!/bin/bash
# main-stream priority A/B on the driver's bench command (edge = encoder tail)
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for P in -1 0 -1 0 -1 0; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --main-priority=$P $OFF > gpurun_out/r04w_one.log 2>&1 || { tail -20 gpurun_out/r04w_one.log; exit 1; }
  grep '^{' gpurun_out/r04w_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('main_priority $P', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'edge', round(c['edge_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3))" | tee -a gpurun_out/r04w.log
done
