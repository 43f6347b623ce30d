#!/bin/bash
# round 4: spin vs blocking host wait in the tracker (A/B, two pairs, headline only)
set -o pipefail
mkdir -p gpurun_out
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
for rep in 1 2; do
for spin in 1 0; do
  S3_SPIN_SYNC=$spin timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04h_one.log 2>&1 || { tail -20 gpurun_out/r04h_one.log; exit 1; }
  grep '^{' gpurun_out/r04h_one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('spin=$spin', round(d['value'],1), round(d['ms_per_step'],3), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), d['frame_breakdown']['decode_ahead'])"
done
done
timeout -k 10 400 python3 -m tools.gemm_ceiling --shapes 768x768x768x2,768x2304x768x2,768x3072x768x2,768x768x3072x2,768x1536x768x2,1536x768x768x2,1536x3072x768x2,1536x768x3072x2 > gpurun_out/r04h_small_gemm.log 2>&1 || { tail -20 gpurun_out/r04h_small_gemm.log; exit 1; }
grep -v WRONG gpurun_out/r04h_small_gemm.log | grep torch
timeout -k 10 300 python3 -m tools.bench_attn > gpurun_out/r04h_attn.log 2>&1 || { tail -20 gpurun_out/r04h_attn.log; exit 1; }
grep " us " gpurun_out/r04h_attn.log
