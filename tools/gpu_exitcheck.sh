set -e
mkdir -p gpurun_out/exitcheck
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exitcheck/c -o c -- python -u tools/exit_probe.py all > gpurun_out/exitcheck/c.log 2>&1 && echo rc=0
