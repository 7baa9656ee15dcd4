# GPU parity suite (pytest -m gpu) with a per-test timeout; log under gpurun_out/.
# usage: bash tools/gpu_tests.sh [tag] [pytest args...]
set -o pipefail
tag=${1:-run}; shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
  > gpurun_out/pytest_gpu_${tag}.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_${tag}.log
exit $rc
