# after the bulk scenario upload: full GPU parity, then the C5-shape line (wall incl. upload)
set -e
mkdir -p gpurun_out/up
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/up/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/up/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/up/pytest_gpu.log
timeout -k 10 400 python -u bench.py --scenarios 512 --steps 2 --warmup 1 --no-traffic > gpurun_out/up/c5.json 2> gpurun_out/up/c5.err || { tail -20 gpurun_out/up/c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/up/c5.json')); print('C5', '%.3g' % d['value'], 'evals/s', round(d['ms_per_step'],2), 'ms device', round(d['wall_ms_per_step_incl_upload'],1), 'ms wall')"
