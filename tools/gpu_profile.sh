# Round-1 measurement: the default bench line (CPU baseline + live PMC traffic), then the
# rocprofv3 kernel-trace stats of the same workload.  Stops at the first failing step.
set -e
mkdir -p gpurun_out/prof_r1
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/prof_r1/bench.json 2> gpurun_out/prof_r1/bench.err
cat gpurun_out/prof_r1/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1/kt -o kt -- python -u bench.py --no-cpu --no-traffic > gpurun_out/prof_r1/kt.log 2>&1
cat gpurun_out/prof_r1/kt/kt_kernel_stats.csv
