set -e
mkdir -p gpurun_out/st
rm -f gpurun_out/st/*.bin
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for w in ${SWEEP:-2 8 20 64}; do
  KSS_SHARDS=$w KSS_STAMPS_FILE=gpurun_out/st/w$w.bin timeout -k 10 120 python -u bench.py --steps 1 --warmup 0 --pods 2000 --no-cpu > gpurun_out/st/w$w.json
done
python tools/stamps.py gpurun_out/st/*.bin
for f in gpurun_out/st/*.json; do python -c "import json,sys; d=json.load(open('$f')); print(d['geometry'], round(d['pods_per_s']), 'pods/s')"; done
