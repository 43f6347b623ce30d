#!/bin/bash
# kernel trace of the headline frame loop after the aux-stream render:
# whole-run and timed-window summaries, per-queue breakdown
set -o pipefail
O=gpurun_out/r06rp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-pairs --no-kprof --no-map --no-backend --no-e2e --no-live > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
grep '^{' $O/bench_prof.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']
print('prof run', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'frames', d['frame_breakdown']['tracked'])"
python -m tools.rocprof_summary gpurun_out/prof/run_results.db > $O/rocprof_summary.txt 2>&1
python -m tools.rocprof_summary gpurun_out/prof/run_results.db --last-ms 110 > $O/rocprof_summary_timed.txt 2>&1
python -m tools.rocprof_queues gpurun_out/prof/run_results.db --last-ms 90 --frames 16 > $O/queues.txt 2>&1
rm -rf gpurun_out/prof
head -50 $O/queues.txt
