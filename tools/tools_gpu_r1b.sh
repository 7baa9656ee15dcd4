set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -50 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest ok"
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
for w in 1 4 8 16 20 32 64; do KSS_SHARDS=$w timeout -k 10 120 python -u bench.py --steps 2 --warmup 1 --pods 3000 --no-cpu >> gpurun_out/sweep.jsonl 2>>gpurun_out/bench.err; done
python - <<'PY'
import json
for l in open("gpurun_out/sweep.jsonl"):
    d=json.loads(l); print(d["geometry"], round(d["pods_per_s"]), "pods/s", round(d["value"]/1e6,1), "Mevals/s")
PY
