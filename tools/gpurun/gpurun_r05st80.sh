#!/bin/bash
# round 5: stall watch over 80-frame windows (S3_STALL_TRACE: stacks of every
# thread when an issue phase of a step exceeds 3 ms)
set -o pipefail
D=gpurun_out/r05st80
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
: > $D/watch.log
for n in 1 2 3; do
  S3_STALL_TRACE=3 S3_HOST_PHASES=1 timeout -k 10 300 python3 bench.py --steps 80 --warmup 5 $OFF > $D/one.log 2> $D/err_$n.log || { tail -20 $D/err_$n.log; exit 1; }
  grep '^{' $D/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
h=c['host_step_ms']; k=max(range(len(h)), key=lambda i: h[i])
print('run $n', round(d['value'],1), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'big_gaps', c['big_gaps'], 'worst step', k, h[k], 'phases', c['host_phases_ms'].get(str(k)))" | tee -a $D/watch.log
  echo "run $n stack dumps: $(grep -c 'most recent call first' $D/err_$n.log || true)" | tee -a $D/watch.log
done
