# Node-axis sharding (C4 shape): GPU parity (world 1 in-process, 2-4 gloo ranks sharing
# cuda:0), then the node-axis bench line at 1 GPU and its rocprofv3 kernel stats.
set -e
mkdir -p gpurun_out/axis
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_nodeaxis.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/axis/pytest.log 2>&1 || { tail -60 gpurun_out/axis/pytest.log; exit 1; }
tail -3 gpurun_out/axis/pytest.log
timeout -k 10 300 python -u bench.py --node-axis --steps 2 --warmup 1 > gpurun_out/axis/bench.json 2> gpurun_out/axis/bench.err || { tail -30 gpurun_out/axis/bench.err; exit 1; }
cat gpurun_out/axis/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/axis/kt -o kt -- python -u bench.py --node-axis --steps 1 --warmup 0 --pods 5000 > gpurun_out/axis/kt.log 2>&1
cat gpurun_out/axis/kt/kt_kernel_stats.csv
