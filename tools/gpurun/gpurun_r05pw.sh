#!/bin/bash
# round 5: the driver command on a fresh box with bench.py's own prewarm (first process)
set -o pipefail
mkdir -p gpurun_out/r05pw
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for r in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05pw/one_$r.log 2> gpurun_out/r05pw/err.log || { tail -20 gpurun_out/r05pw/err.log; exit 1; }
  grep '^{' gpurun_out/r05pw/one_$r.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('run $r', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [(g['frame'], round(g['gap_ms'],2)) for g in c['big_gaps']], 'live', round(d['live_camera']['frames_per_s'],1), 'c3', round(d['raster_c3']['fwd_ms'],3))"
done
