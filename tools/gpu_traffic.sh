# C5-shape and C4-shape bench lines with live PMC traffic (FETCH_SIZE / WRITE_SIZE passes)
set -e
mkdir -p gpurun_out/tr
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --scenarios 512 --steps 2 --warmup 1 > gpurun_out/tr/c5.json 2> gpurun_out/tr/c5.err || { tail -20 gpurun_out/tr/c5.err; exit 1; }
cat gpurun_out/tr/c5.json
timeout -k 10 400 python -u bench.py --node-axis --steps 2 --warmup 1 > gpurun_out/tr/c4.json 2> gpurun_out/tr/c4.err || { tail -20 gpurun_out/tr/c4.err; exit 1; }
cat gpurun_out/tr/c4.json
