# k_spread paths: parity (C3 / C4 full size, fuzz, split), then the C4 and C3 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_spread.py tests/test_gpu_split.py tests/test_gpu_edge_fixtures.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_spread.log 2>&1 || { tail -30 gpurun_out/pytest_spread.log; exit 1; }
tail -2 gpurun_out/pytest_spread.log
timeout -k 10 400 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4.json 2> gpurun_out/c4.err || exit $?
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu --no-traffic > gpurun_out/c3.json 2> gpurun_out/c3.err || exit $?
for f in gpurun_out/c4.json gpurun_out/c3.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['pods_per_s']), round(d['us_per_pod'],2), d['geometry'])"; done
