#!/bin/bash
# The k_spread lines: C4 (one GPU, no CPU leg) and C3 (with its CPU baseline).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config 4 --no-traffic --no-cpu > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
timeout -k 10 400 python -u bench.py --config 3 --no-traffic > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
for f in gpurun_out/bench_c4.json gpurun_out/bench_c3.json; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['pods_per_s']), round(d['us_per_pod'], 3))"
done
