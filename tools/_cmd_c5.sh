T=$1
bash tools/ab_run.sh $T base
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_split.py tests/test_gpu_spread.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/${T}_tests.log)"; [ $rc -eq 0 ] || exit 1
bash tools/gpurecipe.sh $T c5 c3 c1
