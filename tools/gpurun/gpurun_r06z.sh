#!/bin/bash
# round-6 profiles: rocprofv3 kernel trace of the bench, PMC traffic of the
# network on the bench's timed composition and of the C3 raster, then two
# driver-command benches (default pooled streams) reading the new summary
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-pairs --no-kprof --no-map --no-backend --no-e2e > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
python -m tools.rocprof_summary gpurun_out/prof/run_results.db > $O/rocprof_summary.txt 2>&1
python -m tools.rocprof_summary gpurun_out/prof/run_results.db --last-ms 110 > $O/rocprof_summary_timed.txt 2>&1
cp gpurun_out/prof/run_kernel_stats.csv $O/ 2>/dev/null || find gpurun_out/prof -name '*kernel_stats.csv' -exec cp {} $O/ \;
rm -rf gpurun_out/prof
echo "prof done"
rm -rf $O/f $O/w
MIX="--kb 8 --mix 40,5,18,4"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f -o run -- python3 -m tools.pmc_traffic run --reps 2 $MIX > $O/pmc_f.txt 2>&1 || { tail -5 $O/pmc_f.txt; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w -o run -- python3 -m tools.pmc_traffic run --reps 2 $MIX > $O/pmc_w.txt 2>&1 || { tail -5 $O/pmc_w.txt; exit 1; }
python -m tools.pmc_traffic summarize $O/f $O/w --reps 2 $MIX --out $O/r06_pmc_traffic.json > $O/pmc_summary.txt 2>&1 || { tail -5 $O/pmc_summary.txt; exit 1; }
find $O -name '*.csv' -size +2M -delete
echo "network pmc done"
rm -rf $O/rf $O/rw
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/rf -o run -- python3 -m tools.pmc_traffic run --workload raster > $O/rpmc_f.txt 2>&1 || { tail -5 $O/rpmc_f.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/rw -o run -- python3 -m tools.pmc_traffic run --workload raster > $O/rpmc_w.txt 2>&1 || { tail -5 $O/rpmc_w.txt; exit 1; }
python -m tools.pmc_traffic summarize $O/rf $O/rw --workload raster --out $O/r06_raster_pmc.json > $O/rpmc_summary.txt 2>&1
find $O -name '*.csv' -size +2M -delete
echo "raster pmc done"
cp $O/r06_pmc_traffic.json profiles/r06_pmc_traffic.json
for i in 1 2; do
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2> $O/bench$i.err || { tail -20 $O/bench$i.err; exit 1; }
grep '^{' $O/bench$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['critical_path']; r=d['roofline']; iw=r.get('in_window',{})
print('bench$i', round(d['value'],1), 'net', round(c['main_network_ms'],3), 'other', round(c['main_other_ms'],3), 'idle', round(c['main_idle_ms'],3), 'gaps', [round(g['gap_ms'],2) for g in c['big_gaps']], 'frac', round(r['frac'],4), 'iw', round(iw.get('frac',0),4), 'traffic', r.get('traffic'), round(r.get('traffic_over_algorithmic') or 0,3), 'c3', round(d['raster_c3']['fwd_ms'],3), 'be', round(d['fps_with_backend'],1))"
done
