#!/bin/bash
# rocprofv3 kernel summaries of the C3 and C4 bench runs (k_spread).
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -o c3 -- \
  python3 $R/bench.py --config 3 --inner --steps 3 --warmup 1 > $R/gpurun_out/c3_inner.json 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -o c4 -- \
  python3 $R/bench.py --config 4 --inner --steps 3 --warmup 1 > $R/gpurun_out/c4_inner.json 2>&1 || exit $?
