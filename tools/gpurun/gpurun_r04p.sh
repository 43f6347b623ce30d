#!/bin/bash
# bimodal main-stream idle: per-frame idle gaps over repeated runs
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for CFG in PYTORCH_HIP_ALLOC_CONF=expandable_segments:True S3_A=0 PYTORCH_HIP_ALLOC_CONF=expandable_segments:True S3_A=0 PYTORCH_HIP_ALLOC_CONF=expandable_segments:True S3_A=0; do
  env ${CFG:-S3_X=0} timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04p_one.log 2>&1 || { tail -20 gpurun_out/r04p_one.log; exit 1; }
  grep '^{' gpurun_out/r04p_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('$CFG', round(d['value'],1), 'idle', round(c['main_idle_ms'],3), c['idle_gaps_ms']); print('   host', c['host_step_ms'], 'segments', c['segments_allocated'])" | tee -a gpurun_out/r04p3.log
done
