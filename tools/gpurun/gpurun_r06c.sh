#!/bin/bash
# B-direct tiles integrated: op tests, a re-tuning bench run that writes the
# new tuning database, then the driver command with that database
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py -x -q --timeout 300 --timeout-method thread -k "bdirect or split_k_and_tiles or pp_tiles or mf16 or rope_epilogue" > $O/ops_tests.log 2>&1 || { tail -30 $O/ops_tests.log; exit 1; }
tail -1 $O/ops_tests.log
S3_GEMM_TUNE_DB= S3_GEMM_TUNE_DB_SAVE=$O/tune_gfx950.json S3_GEMM_TUNE_LOG=1 timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_tune.log 2> $O/bench_tune.err || { tail -20 $O/bench_tune.err; exit 1; }
ls -la $O/tune_gfx950.json
S3_GEMM_TUNE_DB=$O/tune_gfx950.json timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
for f in bench_tune bench; do grep '^{' $O/$f.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']
print('$f', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'dense', round(r['ms_per_frame'],3), 'frac', round(r['frac'],4), {k: round(v,3) for k,v in r['trace_ms_per_frame'].items()})"; done
