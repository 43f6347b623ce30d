# A/B of the encoder lookahead batch in one box run (headline leg only)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/encb_ab.log
for kb in 1 2 4 1 2 4; do
  timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-pairs --no-backend --no-map --no-c3 --no-kprof --enc-batch $kb > gpurun_out/encb_$kb.log 2>&1 || { tail -20 gpurun_out/encb_$kb.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/encb_$kb.log') if l.startswith('{')][-1]); print('enc_batch', $kb, round(d['value'],2), 'frames/s', round(d['ms_per_step'],3), 'ms')" | tee -a gpurun_out/encb_ab.log
done
