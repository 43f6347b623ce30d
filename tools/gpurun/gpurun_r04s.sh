#!/bin/bash
# host phases of the stalled step
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for CFG in S3_RESERVE=1 S3_RESERVE=0 S3_RESERVE=1 S3_RESERVE=0 S3_RESERVE=1 S3_RESERVE=0; do
  env $CFG S3_HOST_PHASES=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04s_one.log 2>&1 || { tail -20 gpurun_out/r04s_one.log; exit 1; }
  grep '^{' gpurun_out/r04s_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
h=c['host_step_ms']; k=max(range(len(h)), key=lambda i: h[i] if h[i] > 9 else 0)
print('$CFG', round(d['value'],1), c['segments_allocated'], 'worst step', k, h[k], 'phases', c['host_phases_ms'].get(str(k)))" | tee -a gpurun_out/r04s.log
done
