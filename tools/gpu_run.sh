# One GPU session, steps chained with && and each under its own time limit.
#   tools/gpu_run.sh TAG STEP...   STEP in: tests spread smoke bench stamps prof pmc c3 c5 axis
# Output under gpurun_out/TAG/.  Stops at the first failing step.
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ;;
    spread) KSS_TRACE_PATH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_spread.py tests/test_gpu_scale.py -k "spread or c3 or c4" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_spread.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench)  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err ;;
    stamps) rm -f $OUT/*.bin; KSS_STAMPS_FILE=$OUT/simple_c2.bin timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --pods 2000 --no-cpu --no-traffic --no-latency > /dev/null && python tools/stamps.py $OUT/*.bin > $OUT/stamps.txt ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python -u bench.py --no-cpu --no-traffic > $OUT/kt.log 2>&1 ;;
    c3)     timeout -k 10 300 python -u bench.py --config 3 --no-traffic --no-cpu > $OUT/c3.json 2> $OUT/c3.err ;;
    c3stamps) rm -f $OUT/general_c3.bin; KSS_STAMPS_FILE=$OUT/general_c3.bin timeout -k 10 120 python -u bench.py --config 3 --steps 1 --warmup 0 --pods 1000 --no-cpu --no-traffic --no-latency > /dev/null && python tools/stamps.py $OUT/general_c3.bin > $OUT/c3_stamps.txt ;;
    c3prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3kt -o kt -- python -u bench.py --config 3 --pods 2000 --no-cpu --no-traffic > $OUT/c3kt.log 2>&1 ;;
    coopprof) KSS_COOP_LAUNCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/coopkt -o kt -- python -u bench.py --config 3 --pods 500 --steps 1 --warmup 0 --no-cpu --no-traffic > $OUT/coopkt.log 2>&1; echo "coop rc=$?" >> $OUT/coopkt.log ;;
    perpod) timeout -k 10 300 python -u bench.py --per-pod > $OUT/perpod.json 2> $OUT/perpod.err ;;
    c5)     timeout -k 10 300 python -u bench.py --scenarios 512 --no-traffic > $OUT/c5.json 2> $OUT/c5.err ;;
    axis)   timeout -k 10 300 python -u bench.py --node-axis --no-traffic > $OUT/axis.json 2> $OUT/axis.err ;;
    sweep)  for nps in ${SWEEP_NPS:-64 96 128 192 256}; do
              KSS_NODES_PER_SHARD=$nps timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-traffic > $OUT/sweep_n$nps.json 2>> $OUT/sweep.err
              python -c "import json,sys; d=json.load(open('$OUT/sweep_n$nps.json')); print('nps', $nps, d['geometry'], round(d['pods_per_s']), 'pods/s', round(d['us_per_pod'],3), 'us/pod')" >> $OUT/sweep.txt
            done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
