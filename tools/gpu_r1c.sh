# Round-1 re-measure of the latest kernels: GPU parity, smoke, default bench line
# (CPU baseline + live PMC traffic), rocprofv3 kernel stats, other configs.
set -e
mkdir -p gpurun_out/r1c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1c/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r1c/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r1c/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1c/smoke.log 2>&1
cat gpurun_out/r1c/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r1c/bench.json 2> gpurun_out/r1c/bench.err
cat gpurun_out/r1c/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1c/kt -o kt -- python -u bench.py --no-cpu --no-traffic > gpurun_out/r1c/kt.log 2>&1
cat gpurun_out/r1c/kt/kt_kernel_stats.csv
for c in 1 3; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-traffic > gpurun_out/r1c/bench_c$c.json 2> gpurun_out/r1c/bench_c$c.err
  cat gpurun_out/r1c/bench_c$c.json
done
