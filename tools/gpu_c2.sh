# C2 headline: parity of the k_simple paths, then the default bench line (N=1) with its stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_edge_fixtures.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_c2.log 2>&1 || { tail -30 gpurun_out/pytest_c2.log; exit 1; }
tail -3 gpurun_out/pytest_c2.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-traffic --no-cpu > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
cat gpurun_out/bench_c2.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['pods_per_s'], d['us_per_pod'], d['roofline']['latency'])"
