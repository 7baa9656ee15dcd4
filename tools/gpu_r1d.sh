# Round-1 closing measurement: full GPU parity, smoke, default bench line (CPU baseline +
# live PMC traffic) with its rocprofv3 stats, then the C5-shape sweep and the C4-shape
# node-axis lines with their stats.  Stops at the first failing step.
set -e
mkdir -p gpurun_out/r1d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r1d/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/r1d/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r1d/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1d/smoke.log 2>&1
cat gpurun_out/r1d/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r1d/bench.json 2> gpurun_out/r1d/bench.err
cat gpurun_out/r1d/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1d/kt -o kt -- python -u bench.py --no-cpu --no-traffic > gpurun_out/r1d/kt.log 2>&1
timeout -k 10 300 python -u bench.py --scenarios 512 --steps 2 --warmup 1 > gpurun_out/r1d/c5.json 2> gpurun_out/r1d/c5.err
cat gpurun_out/r1d/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1d/kt5 -o kt -- python -u bench.py --scenarios 512 --steps 1 --warmup 0 > gpurun_out/r1d/kt5.log 2>&1
timeout -k 10 300 python -u bench.py --node-axis --steps 2 --warmup 1 > gpurun_out/r1d/c4.json 2> gpurun_out/r1d/c4.err
cat gpurun_out/r1d/c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1d/kt4 -o kt -- python -u bench.py --node-axis --steps 1 --warmup 0 --pods 5000 > gpurun_out/r1d/kt4.log 2>&1
echo r1d done
