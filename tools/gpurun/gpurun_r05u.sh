#!/bin/bash
# round 5: diagnostic A/B: speculative world records / render left out of
# the tracked frame (where do the main-stream gaps come from)
set -o pipefail
mkdir -p gpurun_out/r05u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
for n in 1 2; do
  for S in none world render world,render; do
    S3_DIAG_SKIP=$S timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05u/one.log 2>&1 || { tail -20 gpurun_out/r05u/one.log; exit 1; }
    grep '^{' gpurun_out/r05u/one.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('skip=$S run $n', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3))" | tee -a gpurun_out/r05u/ab.log
  done
done
S3_DIAG_SKIP=world timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05u/prof -o run -- python3 bench.py --steps 30 --warmup 5 $OFF > gpurun_out/r05u/prof.log 2>&1 || exit 1
python -m tools.rocprof_timeline gpurun_out/r05u/prof/run_results.db --last-ms 60 --gaps 15 > gpurun_out/r05u/timeline_noworld.txt 2>&1
rm -f gpurun_out/r05u/prof/run_results.db
