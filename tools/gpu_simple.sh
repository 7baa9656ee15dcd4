# GPU parity tests, then a C2 bench line for the compact kernel across shard sizes and
# one for the general kernel.
set -e
mkdir -p gpurun_out/sw
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for nps in ${SWEEP:-128 256 512 1024}; do
  KSS_NODES_PER_SHARD=$nps timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/sw/n$nps.json
  python -c "import json; d=json.load(open('gpurun_out/sw/n$nps.json')); print('nps=$nps', d['roofline']['kernel'], d['geometry'], round(d['pods_per_s']), 'pods/s', round(d['kernel_ms_per_step'],1), 'ms')"
done
KSS_NO_SIMPLE=1 timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/sw/general.json
python -c "import json; d=json.load(open('gpurun_out/sw/general.json')); print('general', d['roofline']['kernel'], d['geometry'], round(d['pods_per_s']), 'pods/s')"
