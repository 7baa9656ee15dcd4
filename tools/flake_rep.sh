set -o pipefail
for i in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py -m gpu -k 'spread or split' -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4h_$i.log 2>&1; rc=$?
  echo "rep $i rc=$rc $(tail -1 gpurun_out/r4h_$i.log) $(grep -o 'Failed: run [0-9]*: mismatching pods per part \[\[[0-9, ]*' gpurun_out/r4h_$i.log | head -1)"
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu --no-traffic > gpurun_out/r4h_c4.json 2> gpurun_out/r4h_c4.err && tail -c 200 gpurun_out/r4h_c4.json
