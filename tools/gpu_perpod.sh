# per-pod API: parity of every eval_pod user, then the per-pod bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_fixtures.py tests/test_gpu_portimage.py tests/test_gpu_preemption.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_perpod.log 2>&1 || { tail -30 gpurun_out/pytest_perpod.log; exit 1; }
tail -2 gpurun_out/pytest_perpod.log
timeout -k 10 300 python -u bench.py --per-pod > gpurun_out/perpod.json 2> gpurun_out/perpod.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/perpod.json').read().strip().splitlines()[-1]); print(round(d['value']), d['eval_us']['median'], d['eval_slim_us']['median'], d['commit_us']['median'], d['eval_device_ms_last'])"
