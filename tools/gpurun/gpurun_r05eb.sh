#!/bin/bash
# round 5: headline frame rate against the timed window length (20 / 40 / 80 frames)
set -o pipefail
mkdir -p gpurun_out/r05eb
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
for st in 20 40 80 20; do
  timeout -k 10 300 python3 bench.py --steps $st --warmup 5 $OFF > gpurun_out/r05eb/one.log 2>&1 || { tail -20 gpurun_out/r05eb/one.log; exit 1; }
  grep '^{' gpurun_out/r05eb/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; f=d['frame_breakdown']
print('steps $st', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3), 'kf', f['keyframes'], 'gn', f['gn_iters_avg'], 'da', f['decode_ahead'], 'big', c['big_gaps'])" | tee -a gpurun_out/r05eb/ab.log
done
