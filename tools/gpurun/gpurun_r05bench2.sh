#!/bin/bash
# round 5: the driver's bench command twice on one box (final numbers)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for r in b c; do
  s0=$(date +%s)
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_final_bench_$r.log 2> gpurun_out/r05_final_bench_$r.err || { tail -20 gpurun_out/r05_final_bench_$r.err; exit 1; }
  echo "run $r driver bench wall $(( $(date +%s) - s0 )) s"
  grep '^{' gpurun_out/r05_final_bench_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']
print('$r', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', c['big_gaps'], 'frac', round(r['frac'],4), 'traffic/alg', round(r['traffic_over_algorithmic'] or 0,2), 'c3', round(d['raster_c3']['fwd_ms'],3), 'live', round(d['live']['frames_per_s'],1) if d.get('live') else None, 'e2e', round(d.get('end_to_end_fps') or 0,1))"
done
