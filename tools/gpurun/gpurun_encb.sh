set -o pipefail
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.Stream.priority_range())"
for cfg in "1" "1 --main-priority -1" "1" "1 --main-priority -1" "2" "2 --main-priority -1"; do
set -- $cfg; k=$1; shift
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-c3 --no-pairs --no-kprof --steps 80 --enc-batch $k "$@" > gpurun_out/bench_k.log 2>&1 || { tail -20 gpurun_out/bench_k.log; exit 1; }
python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_k.log') if l.startswith('{')][-1]); print('$cfg', d['value'], d['ms_per_step'])"
done
