#!/bin/bash
# round 5: main-chain priority x encoder lookahead, 20- and 80-frame windows
set -o pipefail
D=gpurun_out/r05prio
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
: > $D/watch.log
for rep in 1 2; do
for cfg in "-1 8 8" "0 8 8" "0 4 12"; do
  set -- $cfg
  for st in 20 80; do
    timeout -k 10 300 python3 bench.py --steps $st --warmup 5 --main-priority $1 --enc-batch $2 --enc-ahead $3 $OFF > $D/one.log 2>&1 || { tail -20 $D/one.log; exit 1; }
    grep '^{' $D/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('prio $1 kb $2 ahead $3 steps $st', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'ngaps', len(c['big_gaps']))" | tee -a $D/watch.log
  done
done
done
