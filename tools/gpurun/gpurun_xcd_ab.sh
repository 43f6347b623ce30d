# A/B of the 2-D XCD tile partition (S3_GEMM_XCD=1 disables it): tests, headline bench x2 each, PMC traffic each
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_net_ops.py tests/test_net.py tests/test_n1.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_xcd.log 2>&1 || { tail -30 gpurun_out/t_xcd.log; exit 1; }
tail -1 gpurun_out/t_xcd.log
: > gpurun_out/xcd_ab.log
for v in 0 1 0 1; do
  S3_GEMM_XCD=$v timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-pairs --no-backend --no-map --no-c3 > gpurun_out/bx_$v.log 2>&1 || { tail -20 gpurun_out/bx_$v.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bx_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('xcd_flags', $v, round(d['value'],2), 'frames/s', 'gemm.dense', round(r['ms_per_frame'],3), 'ms/frame', 'frac', round(r['frac'],4), 'trace', {k: round(x,3) for k,x in r['trace_ms_per_frame'].items()})" | tee -a gpurun_out/xcd_ab.log
done
bash tools/gpurun/gpurun_traffic.sh && cp gpurun_out/traffic/traffic.json gpurun_out/traffic_xcd0.json
S3_GEMM_XCD=1 bash tools/gpurun/gpurun_traffic.sh && cp gpurun_out/traffic/traffic.json gpurun_out/traffic_xcd1.json
python -c "
import json
for v in (0, 1):
    d = json.load(open(f'gpurun_out/traffic_xcd{v}.json'))['families']
    print('xcd_flags', v, {k: round(x['bytes_per_frame'] / 1e9, 3) for k, x in d.items() if k.startswith('gemm')}, 'GB/frame')
" | tee -a gpurun_out/xcd_ab.log
