#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r05o
S3_PLAN_BRANCHES=0 timeout -k 10 200 python3 tools/dbg/branch_dbg.py gpurun_out/r05o/b0.npz > gpurun_out/r05o/b0.log 2>&1; tail -4 gpurun_out/r05o/b0.log
S3_PLAN_BRANCHES=1 timeout -k 10 200 python3 tools/dbg/branch_dbg.py gpurun_out/r05o/b1.npz > gpurun_out/r05o/b1.log 2>&1; tail -4 gpurun_out/r05o/b1.log
DBG_GRAPHS=1 S3_PLAN_BRANCHES=1 timeout -k 10 200 python3 tools/dbg/branch_dbg.py gpurun_out/r05o/b1g.npz > gpurun_out/r05o/b1g.log 2>&1; tail -4 gpurun_out/r05o/b1g.log
python3 -c "
import numpy as np
a=np.load('gpurun_out/r05o/b0.npz'); b=np.load('gpurun_out/r05o/b1.npz')
for k in a.files:
    d=np.abs(a[k]-b[k]).max()
    if d>0: print('DIFF', k, d)
print('compared', len(a.files))
"
