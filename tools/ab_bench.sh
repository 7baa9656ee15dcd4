# bench.py A/B: one line per environment setting.  usage: bash tools/ab_bench.sh TAG "BENCH ARGS" SETTING...
# e.g. bash tools/ab_bench.sh r6j "--config 4" X=0 KSS_SHARDS=224 KSS_THREADS=512
set -o pipefail
tag=$1; args=$2; shift 2
O=gpurun_out; mkdir -p $O
i=0
for v in "$@"; do
  env $v timeout -k 10 300 python -u bench.py $args > $O/${tag}_$i.json 2>/dev/null || exit 1
  echo "$i $v $(python -c "import json; d=json.loads(open('$O/${tag}_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), round(d['ms_per_step'],3), d.get('us_per_pod'), d.get('geometry'))")"
  i=$((i + 1))
done
