#!/bin/bash
# One box session: the spread / split GPU tests in one process per library tag, in order
# (the first process on a fresh box is where the many-chunk split failure showed):
#   bash tools/ab_run.sh <name> <lib tag> [<lib tag> ...]     (tag base = libkss.so)
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
for lib in "$@"; do
  KSS_HANDOFF_LOG=gpurun_out/${T}_${lib}_handoff.txt KSS_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py \
    -m gpu -k 'spread or split' -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_$lib.log 2>&1; rc=$?
  echo "$lib rc=$rc: $(tail -1 gpurun_out/${T}_$lib.log) $(grep -o 'Failed: run [0-9]*: mismatching pods per part \[\[[0-9, ]*\|AssertionError: $\|Mismatched elements.*\|err_msg.*run [0-9]' gpurun_out/${T}_$lib.log | head -2 | tr '\n' ' ')"
  [ -f gpurun_out/${T}_${lib}_handoff.txt ] && head -40 gpurun_out/${T}_${lib}_handoff.txt
  [ $rc -le 1 ] || exit $rc
done
