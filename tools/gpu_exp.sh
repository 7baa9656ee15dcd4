#!/bin/bash
# A/B of experiment builds (make -C csrc exp EXP=<tag> EXP_FLAGS=...; KSS_LIB=<tag>) against
# libkss.so (KSS_LIB=base): parity (PYTEST, on the first tag), then CFG's bench line of each
# build, two interleaved rounds.
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-exp}
first=${LIBS%% *}
KSS_LIB=$first timeout -k 10 600 python -u -m pytest ${PYTEST:-tests/test_gpu_spread.py} -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_exp.log 2>&1 || { tail -30 gpurun_out/pytest_exp.log; exit 1; }
tail -2 gpurun_out/pytest_exp.log
for i in 1 2; do
  for lib in base $LIBS; do
    KSS_LIB=$lib timeout -k 10 300 python -u bench.py --config ${CFG:-3} --steps 3 --warmup 1 --no-cpu --no-traffic \
      > gpurun_out/exp_$lib$i.json 2> gpurun_out/exp_$lib$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/exp_$lib$i.json').read().strip().splitlines()[-1]); print('$lib', round(d['pods_per_s']), round(d['us_per_pod'],3), d['roofline'].get('latency', {}).get('phases_us'))"
  done
done
