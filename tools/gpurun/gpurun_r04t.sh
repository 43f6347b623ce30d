#!/bin/bash
# end-to-end leg: spin vs blocking host waits
set -o pipefail
mkdir -p gpurun_out
OFF="--no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for CFG in S3_SPIN_SYNC=1 S3_SPIN_SYNC=0 S3_SPIN_SYNC=1 S3_SPIN_SYNC=0; do
  env $CFG timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04t_one.log 2>&1 || { tail -20 gpurun_out/r04t_one.log; exit 1; }
  grep '^{' gpurun_out/r04t_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$CFG', round(d['value'],1), 'e2e', round(d['end_to_end_fps'],1), d['end_to_end'].get('keyframes'))" | tee -a gpurun_out/r04t.log
done
