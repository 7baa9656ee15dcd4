# C4 shape on one GPU through the on-chip sharded k_simple (node axis inside the GPU),
# automatic geometry and a shard-size sweep; then GPU parity
set -e
mkdir -p gpurun_out/c4s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c4s/pytest.log 2>&1 || { tail -40 gpurun_out/c4s/pytest.log; exit 1; }
tail -1 gpurun_out/c4s/pytest.log
for nps in 0 782 1024; do
  if [ $nps = 0 ]; then E=""; else E="KSS_NODES_PER_SHARD=$nps"; fi
  env $E timeout -k 10 200 python -u bench.py --config 2 --nodes 100000 --pods 20000 --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/c4s/n$nps.json 2> gpurun_out/c4s/n$nps.err || { tail -5 gpurun_out/c4s/n$nps.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c4s/n$nps.json')); print('nps=$nps', d['roofline']['kernel'], d['geometry'], round(d['pods_per_s']), 'pods/s', round(d['kernel_ms_per_step'],1), 'ms')"
done
timeout -k 10 200 python -u bench.py --no-cpu --no-traffic > gpurun_out/c4s/c2.json
python -c "import json; d=json.load(open('gpurun_out/c4s/c2.json')); print('C2', d['roofline']['kernel'], d['geometry'], round(d['pods_per_s']), 'pods/s')"
