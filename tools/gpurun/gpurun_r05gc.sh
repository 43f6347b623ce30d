#!/bin/bash
# round 5: idle gaps of the critical path beside the host phases of the slowest step
set -o pipefail
D=gpurun_out/r05gc
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
: > $D/watch.log
for st in 80 80 80 80 80 80; do
  timeout -k 10 300 python3 bench.py --steps $st --warmup 5 $OFF > $D/one.log 2>&1 || { tail -20 $D/one.log; exit 1; }
  grep '^{' $D/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; h=c['host_step_ms']
big=c['big_gaps']
print('steps $st', round(d['value'],1), 'idle', round(c['main_idle_ms'],3), 'big', big)
for b in big:
    f=b['frame']
    for k in (f-1, f, f+1):
        if 0 <= k < len(h): print('   step', k, h[k], c['host_phases_ms'].get(str(k)))
" | tee -a $D/watch.log
done
