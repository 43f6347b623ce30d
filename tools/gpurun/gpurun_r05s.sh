#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05s
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
S3_PROFILE_HOST=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05s/out.log 2> gpurun_out/r05s/prof.txt || { tail -20 gpurun_out/r05s/prof.txt; exit 1; }
grep '^{' gpurun_out/r05s/out.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])"
