#!/bin/bash
# packed-FP32 hypothesis: the matching stages and the decode-ahead frontend
# with the library built without v_pk_*_f32 (S3_LIB_VARIANT=_nopk) vs default
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() { env "$@" STRESS_SECONDS=10 timeout -k 10 90 python -u tools/stress_bd_concurrency.py > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }; grep RESULT $O/s.log | sed "s/^/[$*] /"; }
run S3_LIB_VARIANT=_nopk STRESS_SIDE=torchs STRESS_VICTIM=stage_iter
run S3_LIB_VARIANT=_nopk STRESS_SIDE=torchs STRESS_VICTIM=stage_prep
run S3_LIB_VARIANT=_nopk STRESS_SIDE=gemm74 STRESS_VICTIM=match
run STRESS_SIDE=torchs STRESS_VICTIM=stage_iter
S3_LIB_VARIANT=_nopk DIAG_TRIALS=3 timeout -k 10 300 python -u tools/diag_decode_ahead.py > $O/diag_nopk.log 2>&1 || { tail -5 $O/diag_nopk.log; exit 1; }
echo "frontend nopk:"; grep -E "^trial|live !=" $O/diag_nopk.log | cut -c1-160
