# C5 sweep: workgroup size sweep for the one-workgroup-per-scenario k_simple launch
set -e
mkdir -p gpurun_out/c5t
for T in 256 512 1024; do
  KSS_THREADS=$T timeout -k 10 200 python -u bench.py --scenarios 512 --steps 2 --warmup 1 > gpurun_out/c5t/t$T.json 2> gpurun_out/c5t/t$T.err || { tail -20 gpurun_out/c5t/t$T.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5t/t$T.json')); print('threads=$T', round(d['ms_per_step'],2), 'ms', '%.3g' % d['value'], 'evals/s')"
done
