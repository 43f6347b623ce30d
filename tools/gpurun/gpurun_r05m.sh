#!/bin/bash
# round 5: headline-config kernel trace with per-queue breakdown (main / encoder / aux)
set -o pipefail
mkdir -p gpurun_out/r05m
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05m/one.log 2>&1 || { tail -20 gpurun_out/r05m/one.log; exit 1; }
grep '^{' gpurun_out/r05m/one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; print(d['value'], d['ms_per_step'], {k: c[k] for k in ('main_network_ms','main_other_ms','main_idle_ms','edge_ms','encoder_side_stream_ms','big_gaps')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05m/prof -o run -- python3 bench.py --steps 40 --warmup 5 $OFF > gpurun_out/r05m/prof.log 2>&1 || { tail -20 gpurun_out/r05m/prof.log; exit 1; }
python -m tools.rocprof_queues gpurun_out/r05m/prof/run_results.db --last-ms 150 --frames 28 > gpurun_out/r05m/queues.txt 2>&1
python -m tools.rocprof_timeline gpurun_out/r05m/prof/run_results.db --last-ms 150 --gaps 15 > gpurun_out/r05m/timeline.txt 2>&1
rm -f gpurun_out/r05m/prof/run_results.db
head -70 gpurun_out/r05m/queues.txt
