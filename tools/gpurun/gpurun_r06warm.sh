#!/bin/bash
# tile choices tuned warm (no L2/MALL flush between timed launches) vs the cold database
set -o pipefail
O=gpurun_out/r06warm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
S3_GEMM_TUNE_COLD=0 S3_GEMM_TUNE_DB= S3_GEMM_TUNE_DB_SAVE=$O/tune_warm.json S3_GEMM_TUNE_LOG=1 timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_warm.log 2> $O/bench_warm.err || { tail -20 $O/bench_warm.err; exit 1; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_cold.log 2> $O/bench_cold.err || { tail -20 $O/bench_cold.err; exit 1; }
S3_GEMM_TUNE_COLD=0 S3_GEMM_TUNE_DB= S3_GEMM_TUNE_LOG=1 timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_warm2.log 2> $O/bench_warm2.err || { tail -20 $O/bench_warm2.err; exit 1; }
for f in bench_warm bench_cold bench_warm2; do grep '^{' $O/$f.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']; iw=r.get('in_window',{})
print('$f', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'enc', round(c['encoder_side_stream_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'frac', round(r['frac'],4), 'dense', round(r['ms_per_frame'],3), 'iw', round(iw.get('frac',0),4))"; done
