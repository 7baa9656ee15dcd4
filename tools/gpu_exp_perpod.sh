#!/bin/bash
# A/B of an experiment build on the per-pod API line: the whole GPU suite on KSS_LIB=$EXP,
# then bench.py --per-pod on libkss.so and on the experiment build, twice.
set -o pipefail
mkdir -p gpurun_out
KSS_LIB=$EXP timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_exp.log 2>&1 || { tail -30 gpurun_out/pytest_exp.log; exit 1; }
tail -2 gpurun_out/pytest_exp.log
for i in 1 2; do
  for lib in base $EXP; do
    KSS_LIB=$lib timeout -k 10 300 python -u bench.py --per-pod --steps 1 --warmup 1 --no-cpu --no-traffic \
      > gpurun_out/pp_$lib$i.json 2> gpurun_out/pp_$lib$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/pp_$lib$i.json').read().strip().splitlines()[-1]); print('$lib', *(round(d[k]['median'],1) for k in ('eval_us','eval_slim_us','eval_view_us')), round(d['eval_device_ms_last']*1000,1))"
  done
done
