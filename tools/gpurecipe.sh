#!/bin/bash
# Evidence recipes for one gpurun call: bash tools/gpurecipe.sh TAG STEP [STEP ...]
# Every step runs under its own time limit; the first failing step ends the call (no GPU step
# runs after a failure).  Outputs go to gpurun_out/TAG_<step>.*; copy what is judged into profiles/.
#
# steps:
#   tests        pytest -m gpu (whole suite; PYTEST_K narrows it with -k, PYTEST_TIMEOUT per test, default 120 s)
#   svc          the service-grid tests alone (45 s per test)
#   smoke        __graft_entry__.smoke()
#   bench        the default line (C2 + c4_split leg, CPU baseline, PMC traffic, latency)
#   gpus2        bench.py --gpus 2 (on a 1-GPU box: must refuse with "2 GPUs requested")
#   c1 c3 c4     bench.py --config 1 / 3 / 4
#   c5           bench.py --scenarios 512 (C5 share of one GPU)
#   split2       bench.py --split 2 (C4 as two parts on the one GPU)
#   perpod       bench.py --per-pod
#   postfilter   bench.py --postfilter
#   prof_c2 prof_c3 prof_c4 prof_c5 prof_pf prof_pp
#                rocprofv3 --kernel-trace --stats of the matching inner bench run
#   sq_c2 sq_c5 sq_pf  rocprofv3 --pmc SQ counter passes (one pass per group) of the inner run
#   counters     rocprofv3 -L (the counters this box's gfx950 exposes)
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp

prof() {  # prof NAME TIMEOUT bench-args...
  local name=$1 t=$2; shift 2
  (cd /tmp && timeout -k 10 "$t" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${tag}_$name" -o k -- \
    python3 "$R/bench.py" --inner "$@" > "$O/${tag}_$name.json" 2> "$O/${tag}_$name.err")
}

sq() {  # sq NAME bench-args...: one rocprofv3 --pmc pass per counter group
  local name=$1; shift
  local groups=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
                "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
                "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_THREAD_CYCLES_VALU")
  local i=0
  for g in "${groups[@]}"; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$O/${tag}_${name}_pmc$i" -o p -- \
      python3 "$R/bench.py" --inner "$@" > "$O/${tag}_${name}_pmc$i.out" 2>&1) || return $?
    i=$((i + 1))
  done
}

run_step() {
  case $1 in
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout ${PYTEST_TIMEOUT:-120} --timeout-method thread \
             ${PYTEST_K:+-k "$PYTEST_K"} > "$O/${tag}_pytest_gpu.log" 2>&1; local rc=$?
           tail -3 "$O/${tag}_pytest_gpu.log"; return $rc ;;
    svc)   timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -m gpu -x -v --timeout 45 --timeout-method thread \
             > "$O/${tag}_pytest_svc.log" 2>&1; local rc=$?
           tail -3 "$O/${tag}_pytest_svc.log"; return $rc ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/${tag}_smoke.log" 2>&1 ;;
    bench) timeout -k 10 700 python -u bench.py > "$O/${tag}_bench.json" 2> "$O/${tag}_bench.err"; local rc=$?
           tail -c 600 "$O/${tag}_bench.json"; return $rc ;;
    gpus2) timeout -k 10 120 python -u bench.py --gpus 2 > "$O/${tag}_gpus2.out" 2>&1
           local rc=$?; cat "$O/${tag}_gpus2.out"; [ $rc -eq 2 ] ;;
    c1) timeout -k 10 300 python -u bench.py --config 1 --steps 20 --warmup 5 > "$O/${tag}_c1.json" 2> "$O/${tag}_c1.err" ;;
    c3) timeout -k 10 500 python -u bench.py --config 3 > "$O/${tag}_c3.json" 2> "$O/${tag}_c3.err" ;;
    c4) timeout -k 10 600 python -u bench.py --config 4 > "$O/${tag}_c4.json" 2> "$O/${tag}_c4.err" ;;
    c5) timeout -k 10 500 python -u bench.py --scenarios 512 --steps 3 --warmup 1 > "$O/${tag}_c5.json" 2> "$O/${tag}_c5.err" ;;
    split2) timeout -k 10 300 python -u bench.py --split 2 --steps 3 --warmup 1 --no-cpu > "$O/${tag}_split2.json" 2> "$O/${tag}_split2.err" ;;
    perpod) timeout -k 10 300 python -u bench.py --per-pod --steps 1 --warmup 1 > "$O/${tag}_perpod.json" 2> "$O/${tag}_perpod.err" ;;
    postfilter) timeout -k 10 400 python -u bench.py --postfilter --steps 2 --warmup 1 > "$O/${tag}_postfilter.json" 2> "$O/${tag}_postfilter.err" ;;
    prof_c2) prof prof_c2 300 --steps 5 --warmup 1 ;;
    prof_c3) prof prof_c3 300 --config 3 --steps 3 --warmup 1 ;;
    prof_c4) prof prof_c4 400 --config 4 --steps 2 --warmup 1 ;;
    prof_c5) prof prof_c5 300 --scenarios 512 --steps 3 --warmup 1 ;;
    prof_pf) prof prof_pf 300 --postfilter --steps 1 --warmup 1 ;;
    prof_pp) prof prof_pp 300 --per-pod --steps 1 --warmup 1 ;;
    sq_c2) sq sq_c2 --steps 1 --warmup 0 ;;
    sq_c5) sq sq_c5 --scenarios 512 --steps 1 --warmup 0 ;;
    sq_pf) sq sq_pf --postfilter --steps 1 --warmup 0 ;;
    counters) (cd /tmp && timeout -s KILL 60 rocprofv3 -L > "$O/${tag}_counters.txt" 2>&1) ;;
    *) echo "unknown step $1"; return 1 ;;
  esac
}

for st in "$@"; do
  echo "== $st $(date +%T)"
  run_step "$st" || { echo "step $st failed (rc $?)"; exit 1; }
done
echo "== done $(date +%T)"
