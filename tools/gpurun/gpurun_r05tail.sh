#!/bin/bash
# round 5: MFMA 1x1 tail of the DPT head conv: network/op tests, then the conv A/B
set -o pipefail
D=gpurun_out/r05tail
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_net_ops.py tests/test_net.py tests/test_n1.py > $D/tests.log 2>&1
rc=$?; tail -3 $D/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m tools.bench_conv_parts --tail --tiles 51,52,48 --B 1 > $D/conv_tail.log 2>&1 || { tail -5 $D/conv_tail.log; exit 1; }
timeout -k 10 300 python3 -u -m tools.bench_conv_parts --tail --tiles 51,52 --B 2 >> $D/conv_tail.log 2>&1 || { tail -5 $D/conv_tail.log; exit 1; }
grep -v amdgpu.ids $D/conv_tail.log
timeout -k 10 300 python3 -u -m tools.bench_conv_parts --tiles 52,51 --B 1 > $D/conv_plain.log 2>&1 || { tail -5 $D/conv_plain.log; exit 1; }
grep -v amdgpu.ids $D/conv_plain.log
