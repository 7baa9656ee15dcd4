#!/bin/bash
# The C1 line and the C5-share scenario line on the current build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config 1 --no-traffic > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || exit $?
timeout -k 10 400 python -u bench.py --scenarios 512 --no-traffic > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit $?
for f in gpurun_out/bench_c1.json gpurun_out/bench_c5.json; do
  python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('pods_per_s'), d['ms_per_step'])"
done
