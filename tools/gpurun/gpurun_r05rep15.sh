#!/bin/bash
# round 5: the driver's bench command repeated on one box (final tree distribution)
set -o pipefail
mkdir -p gpurun_out/r05rep15
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
: > gpurun_out/r05rep15/runs.log
for r in 1 2 3 4 5; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 15 > gpurun_out/r05rep15/one.log 2> gpurun_out/r05rep15/err.log || { tail -20 gpurun_out/r05rep15/err.log; exit 1; }
  grep '^{' gpurun_out/r05rep15/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('run $r', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'c3', round(d['raster_c3']['fwd_ms'],3), 'frac', round(d['roofline']['frac'],4))" | tee -a gpurun_out/r05rep15/runs.log
done
