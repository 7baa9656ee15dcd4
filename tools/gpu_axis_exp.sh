# k_axis_eval timing experiments: grid cap and the statistics atomics
set -e
mkdir -p gpurun_out/axx
B="python -u bench.py --node-axis --steps 1 --warmup 1 --pods 3000"
for nb in 0 64 128 256; do
  KSS_AXIS_BLOCKS=$nb timeout -k 10 120 $B > gpurun_out/axx/b$nb.json
  python -c "import json; d=json.load(open('gpurun_out/axx/b$nb.json')); print('blocks<=$nb', round(d['us_per_pod'],2), 'us/pod', round(d['roofline']['kernel_us'],2), 'us eval')"
done
KSS_AXIS_NO_FOLD=1 timeout -k 10 120 $B > gpurun_out/axx/nofold.json
python -c "import json; d=json.load(open('gpurun_out/axx/nofold.json')); print('no fold', round(d['roofline']['kernel_us'],2), 'us eval')"
