#!/bin/bash
# encoder lookahead batch sweep on the aux-render tree (headline legs only)
set -o pipefail
O=gpurun_out/r06eb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
n=0
for kb in 8 4 16 8 4 16; do
n=$((n+1))
timeout -k 10 400 python3 bench.py --gpus 1 --steps 32 --warmup 5 --enc-batch $kb --enc-ahead $kb --no-c3 --no-pairs --no-map --no-cpu-baseline --no-backend --no-e2e --no-live --no-kprof --no-in-window > $O/bench$n.log 2> $O/bench$n.err || { tail -20 $O/bench$n.err; exit 1; }
grep '^{' $O/bench$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('kb $kb', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']])"
done
