#!/bin/bash
# split-K fixup: GEMM op tests + network parity, then headline A/B (fixup vs reduce launch)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py tests/test_net.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sktests.log 2>&1 || { tail -40 gpurun_out/sktests.log; exit 1; }
tail -2 gpurun_out/sktests.log
ARGS="--no-cpu-baseline --no-c3 --no-pairs --no-backend --no-map --no-e2e"
: > gpurun_out/skab.log
for i in 1 2; do
  for m in 1 0; do
    S3_GEMM_SKFIX=$m timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/skb.log 2>&1 || { tail -20 gpurun_out/skb.log; exit 1; }
    grep '^{"metric"' gpurun_out/skb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('skfix=$m', round(d['value'],1), round(d['ms_per_step'],3), round(r['ms_per_frame'],3), r['launches_per_frame'], round(r['frac'],4), json.dumps({k: round(v,3) for k,v in r.get('trace_ms_per_frame',{}).items()}))" >> gpurun_out/skab.log
  done
done
cat gpurun_out/skab.log
