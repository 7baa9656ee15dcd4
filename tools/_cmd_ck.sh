T=$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py -m gpu -k 'spread or split' -q -s --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_first.log 2>&1; echo "first rc=$? $(tail -1 gpurun_out/${T}_first.log)"; grep -h "hand-off reloads\|Failed: run\|AssertionError: run" gpurun_out/${T}_first.log | head -5
timeout -k 10 900 python -u -m pytest tests/test_gpu_spread.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_split.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1; echo "tests rc=$? $(tail -1 gpurun_out/${T}_tests.log)"; grep -h "hand-off reloads" gpurun_out/${T}_tests.log | head -5
bash tools/gpurecipe.sh $T c4
