#!/bin/bash
# The spread / split GPU test sequence N times in fresh processes, idle gaps between them
# (is the many-chunk split failure tied to the first process on a box, or to an idle GPU?)
#   bash tools/idle_run.sh <name> <lib tag> <runs> <gap seconds>
set -o pipefail
mkdir -p gpurun_out
T=$1; lib=$2; n=$3; gap=$4
for i in $(seq 1 $n); do
  KSS_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py \
    -m gpu -k 'spread or split' -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_$i.log 2>&1; rc=$?
  echo "$i rc=$rc: $(tail -1 gpurun_out/${T}_$i.log) $(grep -o 'Failed: run [0-9]*: mismatching pods per part \[\[[0-9, ]*\|AssertionError: run.*' gpurun_out/${T}_$i.log | head -2 | tr '\n' ' ')"
  [ $rc -le 1 ] || exit $rc
  [ $i -lt $n ] && sleep $gap
done
exit 0
