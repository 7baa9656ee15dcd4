#!/bin/bash
# rocprofv3 kernel summary of the default (C2) bench run.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o c2 -- \
  python3 $R/bench.py --inner --steps 5 --warmup 1 > $R/gpurun_out/c2_inner.json 2>&1 || exit $?
