# raster parity tests + C3 microbench (x2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_raster.py tests/test_gaussian_map.py tests/test_n1.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_raster.log 2>&1 || { tail -40 gpurun_out/t_raster.log; exit 1; }
tail -2 gpurun_out/t_raster.log
for r in 1 2; do
timeout -k 10 120 python -u -m tools.bench_raster --iters 20 > gpurun_out/raster_c3_$r.log 2>&1 || { tail -20 gpurun_out/raster_c3_$r.log; exit 1; }
tail -3 gpurun_out/raster_c3_$r.log
done
