#!/bin/bash
# which matching stage is corrupted by a concurrent MFMA GEMM (hipBLASLt aggressor)
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { env "$@" STRESS_SECONDS=10 timeout -k 10 90 python -u tools/stress_bd_concurrency.py > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }; grep RESULT $O/s.log; }
for v in prep iter occl refine; do run STRESS_SIDE=torchs STRESS_VICTIM=stage_$v; done
