#!/bin/bash
# One box session: the many-chunk split reproduction with the statistics dump (the first
# process on a fresh box is where it shows), then the whole GPU suite and the smoke test.
set -o pipefail
mkdir -p gpurun_out
KSS_SPREAD_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py \
  tests/test_gpu_split.py -m gpu -k 'spread or split' -s -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4e_dbg.log 2>&1
rc=$?
grep -E 'part . |pod|passed|failed|Failed: run' gpurun_out/r4e_dbg.log | tail -16
[ $rc -le 1 ] || exit $rc
bash tools/gpurecipe.sh r4e tests smoke
