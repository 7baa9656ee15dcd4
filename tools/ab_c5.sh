# C5 A/B: bench.py --scenarios 512 under each environment setting given as an argument
# (e.g. KSS_STATIC_PPB=16); outputs gpurun_out/<tag>_<i>.json.  usage: bash tools/ab_c5.sh TAG SETTING...
set -o pipefail
tag=$1; shift
O=gpurun_out; mkdir -p $O
i=0
for v in "$@"; do
  env $v timeout -k 10 200 python -u bench.py --scenarios 512 --steps 3 --warmup 1 > $O/${tag}_$i.json 2>/dev/null || exit 1
  echo "$i $v $(python -c "import json; d=json.loads(open('$O/${tag}_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), round(d['ms_per_step'],3))")"
  i=$((i + 1))
done
