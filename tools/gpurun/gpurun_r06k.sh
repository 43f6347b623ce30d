#!/bin/bash
# where does bench.py sit silent: all-thread traceback after 100 s
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S3_GEMM_TUNE_LOG=1 timeout -k 10 200 python -u -c "
import faulthandler, sys, runpy
faulthandler.dump_traceback_later(100, exit=True)
sys.argv = ['bench.py', '--gpus', '1', '--steps', '20', '--warmup', '5']
runpy.run_path('bench.py', run_name='__main__')
" > $O/bench.log 2> $O/bench.err; echo "rc=$?"; tail -5 $O/bench.log | cut -c1-200; tail -60 $O/bench.err
