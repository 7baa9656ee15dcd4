#!/bin/bash
# Round-2 evidence: node-axis/limits/preemption GPU tests, the PostFilter bench, the C3
# bench (CPU baseline, PMC traffic, latency) and a C3 rocprofv3 kernel trace.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_limits.py tests/test_gpu_preemption.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/scale.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi  # a test failure is read later; a crash or timeout ends the call
timeout -k 10 300 python -u bench.py --postfilter --steps 2 --cpu-seconds 20 > gpurun_out/postfilter.json 2> gpurun_out/postfilter.err || exit $?
timeout -k 10 400 python -u bench.py --config 3 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o c3 -- \
  python3 $R/bench.py --config 3 --inner --steps 2 --warmup 1 > $R/gpurun_out/c3_inner.json 2>&1
