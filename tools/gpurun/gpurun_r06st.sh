#!/bin/bash
# catch the intermittent host stall: stall watchdog (4 ms) on three driver-command runs
set -o pipefail
O=gpurun_out/r06st
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for i in 1 2 3; do
S3_STALL_TRACE=4 timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
grep '^{' $O/bench$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('run $i', round(d['value'],1), 'gaps', c['big_gaps'], 'host', [round(x,1) for x in c['host_step_ms']][5:10])"
echo "dumps: $(grep -c 'most recent call first' $O/bench$i.err)"
done
