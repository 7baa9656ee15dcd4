set -e
mkdir -p gpurun_out
cd _old
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 100 --timeout-method thread -k "test_schedule_batch_matches_oracle and 3-1500-120-single" > ../gpurun_out/diag.log 2>&1 || { tail -30 ../gpurun_out/diag.log; exit 1; }
tail -3 ../gpurun_out/diag.log
