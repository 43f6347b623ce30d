#!/bin/bash
# round 5: host marks on the device clock around the GN sync
set -o pipefail
mkdir -p gpurun_out/r05w
OFF="--no-e2e --no-pairs --no-backend --no-map --no-c3 --no-cpu-baseline --no-live --no-kprof"
S3_HOST_EVENTS=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $OFF > gpurun_out/r05w/one.log 2>&1 || { tail -20 gpurun_out/r05w/one.log; exit 1; }
grep '^{' gpurun_out/r05w/one.log > gpurun_out/r05w/line.json
python3 - <<'PY'
import json, statistics as S
d = json.load(open('gpurun_out/r05w/line.json'))
c = d['critical_path']; m = c['host_device_marks']
print('fps', round(d['value'], 1), 'other', round(c['main_other_ms'], 3))
keys = sorted(m, key=int)
rows = []
for k in keys:
    ev = dict(m[k])
    nxt = dict(m.get(str(int(k) + 1), []))
    if 'gpu:gn_end' not in ev or 'host:gn_done' not in ev: continue
    g = ev['gpu:gn_end']
    r = {'wake': ev['host:gn_done'] - g}
    for nm in ('host:tracked', 'host:step_end'):
        if nm in ev: r[nm] = ev[nm] - g
    for nm in ('host:step_begin', 'host:delivered', 'host:prefetched', 'host:track_start', 'host:matched', 'chain_start'):
        if nm in nxt: r['next ' + nm] = nxt[nm] - g
    if 'chain_end' in ev: r['chain_end'] = ev['chain_end'] - g
    rows.append(r)
    print(k, {a: round(b, 3) for a, b in r.items()})
print('median ms after this frame GN chunk end:')
for key in rows[0]:
    vals = [r[key] for r in rows if key in r]
    print(f'  {key:24s} {S.median(vals):7.3f}')
PY
