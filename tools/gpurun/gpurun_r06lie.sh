#!/bin/bash
set -o pipefail
O=gpurun_out/r06lie
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { env "$@" STRESS_SECONDS=12 timeout -k 10 90 python -u tools/stress_bd_concurrency.py > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }; grep RESULT $O/s.log; }
run STRESS_SIDE=gemm74 STRESS_VICTIM=lie
run STRESS_SIDE=torchs STRESS_VICTIM=lie
run STRESS_SIDE=enc STRESS_VICTIM=match
