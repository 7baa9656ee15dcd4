# C2 k_simple geometry sweep: nodes per shard x threads
set -e
mkdir -p gpurun_out/c2s
for nps in 64 96 128 160; do
  for T in 64 128; do
    KSS_NODES_PER_SHARD=$nps KSS_THREADS=$T timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/c2s/n${nps}_t$T.json 2> gpurun_out/c2s/n${nps}_t$T.err || { tail -5 gpurun_out/c2s/n${nps}_t$T.err; continue; }
    python -c "import json; d=json.load(open('gpurun_out/c2s/n${nps}_t$T.json')); print('nps=$nps T=$T', d['roofline']['kernel'], d['geometry'], round(d['pods_per_s']), 'pods/s')"
  done
done
