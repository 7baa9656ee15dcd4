set -e
mkdir -p gpurun_out/st
rm -f gpurun_out/st/*.bin
for w in 2 8 20 64; do
  KSS_SHARDS=$w KSS_STAMPS_FILE=gpurun_out/st/w$w.bin timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --pods 1000 --no-cpu > gpurun_out/st/w$w.json
done
python tools/stamps.py gpurun_out/st/*.bin
