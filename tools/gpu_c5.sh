# Scenario sweep parity (k_simple and k_schedule sweeps) and the C5-shape bench lines
set -e
mkdir -p gpurun_out/c5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k scenarios -x -v --timeout 120 --timeout-method thread > gpurun_out/c5/pytest.log 2>&1 || { tail -40 gpurun_out/c5/pytest.log; exit 1; }
tail -2 gpurun_out/c5/pytest.log
for S in 64 512; do
  timeout -k 10 300 python -u bench.py --scenarios $S --steps 2 --warmup 1 > gpurun_out/c5/s$S.json 2> gpurun_out/c5/s$S.err || { tail -20 gpurun_out/c5/s$S.err; exit 1; }
  cat gpurun_out/c5/s$S.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/kt -o kt -- python -u bench.py --scenarios 512 --steps 1 --warmup 0 > gpurun_out/c5/kt.log 2>&1
cat gpurun_out/c5/kt/kt_kernel_stats.csv
