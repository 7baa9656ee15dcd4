#!/bin/bash
# The node-axis evidence (config C4, 100k nodes x 20k pods): the 1-GPU bench line, the
# split-grid lines (1 part; 2 parts on the one GPU), the C3 line (same k_spread code path)
# and the rocprofv3 kernel summary of the C4 bench.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py --config 4 --no-traffic > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
tail -c 300 gpurun_out/bench_c4.json
timeout -k 10 400 python -u bench.py --config 3 --no-traffic > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
timeout -k 10 300 python -u bench.py --split 1 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c4_p1.json 2> gpurun_out/split_c4_p1.err || exit $?
timeout -k 10 300 python -u bench.py --split 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c4_p2.json 2> gpurun_out/split_c4_p2.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o c4 -- \
  python3 $R/bench.py --config 4 --inner --steps 3 --warmup 1 > $R/gpurun_out/c4_inner.json 2>&1 || exit $?
