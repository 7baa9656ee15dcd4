# C2 bench across shard sizes (compact kernel), 1 step each
set -e
mkdir -p gpurun_out/sw
for nps in ${SWEEP:-63 80 100 128}; do
  KSS_NODES_PER_SHARD=$nps timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/sw/n$nps.json
  python -c "import json; d=json.load(open('gpurun_out/sw/n$nps.json')); print('nps=$nps', d['roofline']['kernel'], d['geometry'], round(d['pods_per_s']), 'pods/s', round(d['kernel_ms_per_step'],1), 'ms')"
done
