#!/bin/bash
# A/B on one box: B-direct tiles on (default) vs off (S3_GEMM_BDIRECT=0), x2
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
F="--gpus 1 --steps 20 --warmup 5 --no-c3 --no-pairs --no-backend --no-map --no-e2e --no-live --no-cpu-baseline"
for i in 1 2; do
for v in 1 0; do
S3_GEMM_BDIRECT=$v timeout -k 10 400 python3 bench.py $F > $O/b${v}_$i.log 2> $O/b${v}_$i.err || { tail -20 $O/b${v}_$i.err; exit 1; }
grep '^{' $O/b${v}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']; n=d['network']['kernels']
print('bdirect=$v', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'dense trace', round(r['ms_per_frame'],3), 'launches', round(r['launches_per_frame'],1), 'eager', round(n['gemm.dense']['ms'],3), 'frac', round(r['frac'],4), r['timing'][:30])"
done; done
