#!/bin/bash
# round 4: headline-config kernel trace (device path only) after the refine change
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 $OFF > gpurun_out/r04g_one.log 2>&1 || { tail -20 gpurun_out/r04g_one.log; exit 1; }
grep '^{' gpurun_out/r04g_one.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('critical_path'))"
rm -rf gpurun_out/prof4g
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4g -o run -- python3 bench.py --steps 40 --warmup 5 $OFF > gpurun_out/r04g_prof.log 2>&1 || { tail -20 gpurun_out/r04g_prof.log; exit 1; }
python -m tools.rocprof_timeline gpurun_out/prof4g/run_results.db --last-ms 150 --gaps 15 > gpurun_out/r04g_timeline.txt 2>&1
python -m tools.rocprof_summary gpurun_out/prof4g/run_results.db --last-ms 150 > gpurun_out/r04g_summary_last.txt 2>&1
rm -f gpurun_out/prof4g/run_results.db
head -8 gpurun_out/r04g_timeline.txt
head -45 gpurun_out/r04g_summary_last.txt
