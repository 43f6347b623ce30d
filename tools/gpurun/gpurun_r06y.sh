#!/bin/bash
# the frame-16 main-queue gap: stall watchdog, torch pooled streams vs dedicated
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
n=0
for cfg in "S3_STALL_TRACE=3" "S3_FRAME_STREAMS=0" "X=1" "S3_FRAME_STREAMS=0"; do
n=$((n+1))
env $cfg timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$n.log 2> $O/bench$n.err || { tail -20 $O/bench$n.err; exit 1; }
grep '^{' $O/bench$n.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('$cfg', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', c['big_gaps'], 'host', c['host_step_ms'][8:11])"
done
grep -c "Thread 0x" $O/bench1.err || true
