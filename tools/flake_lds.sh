set -o pipefail
for i in 1 2; do
  KSS_SPREAD_MIN_LDS=${MIN_LDS:-90000} timeout -k 10 300 python -u -m pytest tests/test_gpu_edge_fixtures.py tests/test_gpu_scale.py tests/test_gpu_split.py -m gpu -k 'spread or split' -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r4g_$i.log 2>&1; rc=$?
  echo "minlds rep $i rc=$rc $(tail -1 gpurun_out/r4g_$i.log) $(grep -o 'Failed: run [0-9]*: mismatching pods per part \[\[[0-9, ]*' gpurun_out/r4g_$i.log | head -1)"
  [ $rc -le 1 ] || exit $rc
done
