#!/bin/bash
# Round-2 evidence: C1 and C4 bench lines (CPU baselines for BASELINE.md), rocprofv3
# kernel-trace summaries of C3 (k_spread) and of the PostFilter dry run (k_preempt_*),
# and the PostFilter line with its CPU baseline.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py --config 1 > gpurun_out/c1.json 2> gpurun_out/c1.err || exit $?
timeout -k 10 400 python -u bench.py --config 4 --no-latency > gpurun_out/c4.json 2> gpurun_out/c4.err || exit $?
timeout -k 10 300 python -u bench.py --postfilter --steps 3 --cpu-seconds 20 > gpurun_out/postfilter_cpu.json 2> gpurun_out/postfilter_cpu.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -o c3 -- \
  python3 $R/bench.py --config 3 --inner --steps 2 --warmup 1 > $R/gpurun_out/c3_inner.json 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_pf -o pf -- \
  python3 $R/bench.py --postfilter --steps 1 --no-cpu > $R/gpurun_out/pf_inner.json 2>&1
