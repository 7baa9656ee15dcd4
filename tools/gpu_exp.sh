#!/bin/bash
# A/B of experiment builds against libkss.so, in one box session:
#   make -C kube-scheduler-simulator_amd/csrc exp EXP=<tag> EXP_FLAGS="-D..."   (here, on the CPU)
#   gpurun -- 'LIBS="<tag> ..." CFG=<n|perpod> PYTEST=<tests> bash tools/gpu_exp.sh'
# Parity first (PYTEST on the first tag, default tests/test_gpu_spread.py), then the bench line of
# each build (KSS_LIB=base is libkss.so) in two interleaved rounds: CFG=1..4 runs
# bench.py --config CFG, CFG=perpod runs bench.py --per-pod.
set -o pipefail
mkdir -p gpurun_out
LIBS=${LIBS:-exp}
CFG=${CFG:-3}
first=${LIBS%% *}
KSS_LIB=$first timeout -k 10 600 python -u -m pytest ${PYTEST:-tests/test_gpu_spread.py} -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_exp.log 2>&1 || { tail -30 gpurun_out/pytest_exp.log; exit 1; }
tail -2 gpurun_out/pytest_exp.log
if [ "$CFG" = perpod ]; then mode="--per-pod --steps 1 --warmup 1"; else mode="--config $CFG --steps 3 --warmup 1"; fi
for i in 1 2; do
  for lib in base $LIBS; do
    KSS_LIB=$lib timeout -k 10 300 python -u bench.py $mode --no-cpu --no-traffic --no-c4 \
      > gpurun_out/exp_$lib$i.json 2> gpurun_out/exp_$lib$i.err || exit $?
    python - "$lib" "gpurun_out/exp_$lib$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
if "eval_us" in d:
    print(sys.argv[1], {k: d.get(k) for k in ("eval_us", "eval_view_us", "commit_us")}, d.get("service", {}).get("eval_us"))
else:
    print(sys.argv[1], round(d["pods_per_s"]), round(d["us_per_pod"], 3), (d["roofline"].get("latency") or {}).get("phases_us"))
PY
  done
done
