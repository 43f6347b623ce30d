#!/bin/bash
# round 5: first-run-on-a-fresh-box gap: the tree's files read into the page cache first, then the driver command x3
set -o pipefail
mkdir -p gpurun_out/r05warm
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
find . -type f \( -name '*.so' -o -name '*.py' -o -name '*.json' \) -not -path './gpurun_out/*' -exec cat {} + > /dev/null
python3 -c "import torch, numpy" 2>/dev/null
: > gpurun_out/r05warm/runs.log
for r in 1 2 3; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05warm/one.log 2> gpurun_out/r05warm/err.log || { tail -20 gpurun_out/r05warm/err.log; exit 1; }
  grep '^{' gpurun_out/r05warm/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('run $r', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [(g['frame'], round(g['gap_ms'],2)) for g in c['big_gaps']])" | tee -a gpurun_out/r05warm/runs.log
done
