#!/bin/bash
# round-6 final tree final (aux-stream render, bench names the render stream): full GPU suite, smoke, three driver-command benches
set -o pipefail
O=gpurun_out/r06final4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
grep '^{' $O/bench$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']; iw=r.get('in_window',{})
print('bench$i', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'frac', round(r['frac'],4), 'iw', round(iw.get('frac',0),4), 'c3', round(d['raster_c3']['fwd_ms'],3), 'live', round(d['live_camera']['frames_per_s'],1), 'e2e', round(d['end_to_end_fps'],1), 'be', round(d['fps_with_backend'],1), round(d['fps_with_backend_drained'],1), 'cpu', round(d['cpu_baseline']['value'],3), 'segs', d['critical_path']['segments_allocated'])"
done
