set -e
mkdir -p gpurun_out/st
rm -f gpurun_out/st/*.bin
for nps in ${SWEEP:-63 128}; do
  KSS_NODES_PER_SHARD=$nps KSS_STAMPS_FILE=gpurun_out/st/simple_n$nps.bin timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --pods 2000 --no-cpu --no-traffic > /dev/null
done
python tools/stamps.py gpurun_out/st/*.bin
