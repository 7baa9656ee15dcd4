# split-grid node axis on one GPU: 1 part (on-chip reference), 2 and 4 parts in one process
set -o pipefail
mkdir -p gpurun_out
for p in 1 2; do
  timeout -k 10 300 python -u bench.py --split $p --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c4_p$p.json 2> gpurun_out/split_c4_p$p.err || exit $?
  tail -c 600 gpurun_out/split_c4_p$p.json
done
timeout -k 10 300 python -u bench.py --split 2 --split-recipe 2 --nodes 100000 --pods 20000 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c2_p2.json 2> gpurun_out/split_c2_p2.err || exit $?
timeout -k 10 300 python -u bench.py --split 1 --split-recipe 2 --nodes 100000 --pods 20000 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c2_p1.json 2> gpurun_out/split_c2_p1.err || exit $?
