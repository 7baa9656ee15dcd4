# One GPU session, steps chained with && and each under its own time limit.
#   tools/gpu_run.sh TAG STEP...   STEP in: tests smoke bench stamps prof pmc c3 c5 axis
# Output under gpurun_out/TAG/.  Stops at the first failing step.
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 ;;
    smoke)  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench)  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err ;;
    stamps) rm -f $OUT/*.bin; KSS_STAMPS_FILE=$OUT/simple_c2.bin timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --pods 2000 --no-cpu --no-traffic > /dev/null && python tools/stamps.py $OUT/*.bin > $OUT/stamps.txt ;;
    prof)   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python -u bench.py --no-cpu --no-traffic > $OUT/kt.log 2>&1 ;;
    c3)     timeout -k 10 300 python -u bench.py --config 3 --no-traffic --no-cpu > $OUT/c3.json 2> $OUT/c3.err ;;
    c5)     timeout -k 10 300 python -u bench.py --scenarios 512 --no-traffic > $OUT/c5.json 2> $OUT/c5.err ;;
    axis)   timeout -k 10 300 python -u bench.py --node-axis --no-traffic > $OUT/axis.json 2> $OUT/axis.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
