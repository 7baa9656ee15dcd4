set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --pods 2000 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python -u bench.py --steps 2 --warmup 1 --pods 2000 --no-cpu > gpurun_out/prof.log 2>&1
echo "prof ok"
