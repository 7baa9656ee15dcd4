set -o pipefail
O=gpurun_out; mkdir -p $O
for v in 8 16 32 64; do
  KSS_STATIC_PPB=$v timeout -k 10 200 python -u bench.py --scenarios 512 --steps 3 --warmup 1 > $O/r5z_ppb$v.json 2>/dev/null || exit 1
done
KSS_STATIC_BYTES=4294967296 timeout -k 10 200 python -u bench.py --scenarios 512 --steps 3 --warmup 1 > $O/r5z_4g.json 2>/dev/null || exit 1
(cd /tmp && KSS_STATIC_BYTES=4294967296 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/r5z_prof4g -o k -- python3 $GRAFT_REPO_ROOT/bench.py --inner --scenarios 512 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/r5z_prof4g.json 2>/dev/null)
