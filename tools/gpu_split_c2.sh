# split grid with the default-profile recipe (k_simple, 128 shards in all) at 100k nodes x 20k pods
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --split 1 --split-recipe 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c2r_p1.json 2> gpurun_out/split_c2r_p1.err || exit $?
timeout -k 10 300 python -u bench.py --split 2 --split-recipe 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c2r_p2.json 2> gpurun_out/split_c2r_p2.err || exit $?
for f in gpurun_out/split_c2r_p1.json gpurun_out/split_c2r_p2.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', round(d['pods_per_s']), d['kernel'], d['geometry'])"; done
