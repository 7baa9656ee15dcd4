#!/bin/bash
# Round-2 closing evidence (r2z): full GPU parity, smoke, the default bench line (C2: CPU baseline,
# live PMC traffic, latency roofline) with its rocprofv3 kernel summary, the C3 line, and
# the split-grid node-axis lines (C4 recipe: 1 part, 2 parts on the one GPU).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
bash tools/gpu_tests.sh r2z_full || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
tail -c 400 gpurun_out/bench_default.json
timeout -k 10 400 python -u bench.py --config 3 --no-traffic > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
timeout -k 10 300 python -u bench.py --split 1 --steps 3 --warmup 1 > gpurun_out/split_c4_p1.json 2> gpurun_out/split_c4_p1.err || exit $?
timeout -k 10 300 python -u bench.py --split 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/split_c4_p2.json 2> gpurun_out/split_c4_p2.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o c2 -- \
  python3 $R/bench.py --inner --steps 5 --warmup 1 > $R/gpurun_out/c2_inner.json 2>&1 || exit $?
cd $R
timeout -k 10 400 python -u bench.py --config 4 --no-traffic > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
timeout -k 10 300 python -u bench.py --per-pod --steps 1 --warmup 1 --no-cpu --no-traffic > gpurun_out/perpod.json 2> gpurun_out/perpod.err || exit $?
