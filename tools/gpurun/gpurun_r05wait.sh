#!/bin/bash
# round 5: main-queue gaps beside the device time of the waits on encoder batches (S3_WAIT_EVENTS)
set -o pipefail
D=gpurun_out/r05wait
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
: > $D/watch.log
for st in 80 80 80 80 80 80; do
  S3_WAIT_EVENTS=1 timeout -k 10 300 python3 bench.py --steps $st --warmup 5 $OFF > $D/one.log 2>&1 || { tail -20 $D/one.log; exit 1; }
  grep '^{' $D/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('steps $st', round(d['value'],1), 'idle', round(c['main_idle_ms'],3), 'gaps', [(g['frame'], round(g['gap_ms'],2)) for g in c['big_gaps']], 'enc waits', c.get('encoder_waits'))" | tee -a $D/watch.log
done
