#!/bin/bash
# timed-region encoder plan A/B on the driver's bench command
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for CFG in S3_PLAN_OVERLAP=1 S3_PLAN_OVERLAP=0 S3_PLAN_OVERLAP=1 S3_PLAN_OVERLAP=0 S3_PLAN_OVERLAP=1 S3_PLAN_OVERLAP=0; do
  env $CFG timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04x_one.log 2>&1 || { tail -20 gpurun_out/r04x_one.log; exit 1; }
  grep '^{' gpurun_out/r04x_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('$CFG', round(d['value'],1), 'encodes', d['config'].get('timed_encodes', d.get('timed_encodes')), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'edge', round(c['edge_ms'],3), 'head', c.get('edge_head_ms_total'), 'enc_tail', c.get('enc_tail_ms_total'), 'enc', round(c['encoder_side_stream_ms'],3))" | tee -a gpurun_out/r04x_ab.log
done
