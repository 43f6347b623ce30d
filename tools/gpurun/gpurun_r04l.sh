#!/bin/bash
# one frame of the headline loop kernel by kernel (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export S3_DECODE_EARLY=${S3_DECODE_EARLY:-1}
rm -rf gpurun_out/prof4l
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-kprof --no-live"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof4l -o run -- python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r04l_prof.log 2>&1 || { tail -20 gpurun_out/r04l_prof.log; exit 1; }
python -m tools.rocprof_timeline gpurun_out/prof4l/run_results.db --last-ms 25 --skip-last-ms 3 --list 2000 > gpurun_out/r04l_list.txt 2>&1
rm -f gpurun_out/prof4l/run_results.db
head -3 gpurun_out/r04l_list.txt
