#!/bin/bash
# B-direct split-K: op tests, retune into a new database, GEMM vs hipBLASLt, benches
set -o pipefail
O=gpurun_out/r06s8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests/test_net_ops.py -x -q --timeout 300 --timeout-method thread -k "bdirect or split_k or pp_tiles or mf16" > $O/ops.log 2>&1 || { tail -30 $O/ops.log; exit 1; }
tail -1 $O/ops.log
S3_GEMM_TUNE_DB= S3_GEMM_TUNE_DB_SAVE=$O/tune_gfx950.json S3_GEMM_TUNE_LOG=1 timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_tune.log 2> $O/bench_tune.err || { tail -20 $O/bench_tune.err; exit 1; }
cp $O/tune_gfx950.json splatt3r-slam_amd/splatt3r_amd/tune_gfx950.json
timeout -k 10 300 python -u -m tools.gemm_vs_hipblaslt > $O/blt.log 2>&1 || { tail -5 $O/blt.log; exit 1; }
grep -v amdgpu.ids $O/blt.log
for i in 1 2; do
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
done
for f in bench_tune bench1 bench2; do grep '^{' $O/$f.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']; iw=r.get('in_window',{})
print('$f', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'frac', round(r['frac'],4), 'dense', round(r['ms_per_frame'],3), 'iw', round(iw.get('frac',0),4))"; done
grep -h "gemm-tune" $O/bench_tune.log | grep -c "split [2-8]" || true
grep -h "gemm-tune" $O/bench_tune.log | grep -c "tile 8[01]" || true
