T=$1
bash tools/ab_run.sh $T base || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edge_fixtures.py tests/test_gpu_limits.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/${T}_tests.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/c2_stamps.py 2 0 > gpurun_out/${T}_stamps.txt 2>&1; echo "stamps rc=$?"; cat gpurun_out/${T}_stamps.txt
bash tools/gpurecipe.sh $T bench
