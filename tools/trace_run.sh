#!/bin/bash
# One box session for the many-chunk split diagnosis (tools/split_trace_test.py): the trace
# build as the first process (where the failure showed), then the product suite sequence.
set -o pipefail
mkdir -p gpurun_out
T=${1:-tr}
run() {  # name, env, pytest args...
  local name=$1; shift
  env "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -E '^run [0-9]|passed|failed' gpurun_out/${T}_$name.log | tr '\n' ' ' | cut -c1-900)"
  return $rc
}
PY="timeout -k 10 300 python -u -m pytest -m gpu -s -q --timeout 240 --timeout-method thread -p no:cacheprovider"
run trace KSS_LIB=${LIB:-trace} $PY tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py::test_in_process_parts_match_oracle "tests/test_gpu_split.py::test_parts_over_many_chunks[2-3000-240-30-8]" "tests/test_gpu_split.py::test_parts_over_many_chunks[2-3000-240-31-8]" tools/split_trace_test.py -k 'spread or split or trace or in_process or many_chunks'; rc=$?
[ $rc -le 1 ] || exit $rc
[ -n "$NOPRODUCT" ] && exit $rc
run product KSS_LIB=base $PY tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py -k 'spread or split'; rc=$?
exit $rc
