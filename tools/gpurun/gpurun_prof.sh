#!/bin/bash
# rocprofv3 kernel trace of a short bench run (no CPU leg, no C3, no pairs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-c3 --no-pairs --no-kprof --no-map --no-backend --no-e2e $BENCH_ARGS > gpurun_out/bench_prof.log 2>&1 || exit $?
(python -m tools.rocprof_timeline gpurun_out/prof/run_results.db --last-ms ${WIN_MS:-60} --list ${LIST:-0} --gaps ${GAPS:-0} > gpurun_out/timeline.txt 2>&1)
(python -m tools.rocprof_summary gpurun_out/prof/run_results.db > gpurun_out/prof_summary.txt && python -m tools.rocprof_summary gpurun_out/prof/run_results.db --last-ms ${WIN_MS:-60} > gpurun_out/prof_summary_timed.txt 2>&1)
rm -f gpurun_out/prof/run_results.db
