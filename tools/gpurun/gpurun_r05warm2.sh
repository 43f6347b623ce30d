#!/bin/bash
# round 5: first-run gap: a trivial GPU process first (torch init + one small matmul), then the driver command x2
set -o pipefail
mkdir -p gpurun_out/r05warm2
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python3 -c "import torch; a=torch.randn(4,4,device='cuda'); print(float((a@a).sum())); torch.cuda.synchronize()" > /dev/null 2>&1 || exit 1
: > gpurun_out/r05warm2/runs.log
for r in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05warm2/one.log 2> gpurun_out/r05warm2/err.log || { tail -20 gpurun_out/r05warm2/err.log; exit 1; }
  grep '^{' gpurun_out/r05warm2/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('run $r', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [(g['frame'], round(g['gap_ms'],2)) for g in c['big_gaps']])" | tee -a gpurun_out/r05warm2/runs.log
done
