#!/bin/bash
# round 5: GEMM epilogue operands loaded before the K loop: op / network tests, then the A/B
set -o pipefail
D=gpurun_out/r05epi
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_net_ops.py tests/test_net.py > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m tools.bench_gemm_epi --early > $D/ab.log 2>&1 || { tail -5 $D/ab.log; exit 1; }
grep -v amdgpu.ids $D/ab.log
