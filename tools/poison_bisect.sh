#!/bin/bash
# Which device allocation's initial contents change a k_spread result: one diag_flake run per
# allocation index with only that allocation filled with a byte pattern (KSS_POISON=i).
# usage: bash tools/poison_bisect.sh OUTFILE [max_index]
out=$1; max=${2:-40}
set -o pipefail
: > "$out"
timeout -k 10 120 env KSS_POISON=all python -u tools/diag_flake.py single 1 > "$out.all" 2>&1 || { echo "all-poison run failed" >> "$out"; exit 1; }
n=$(grep -c "kss poison: allocation" "$out.all")
echo "allocations: $n" >> "$out"
grep "kss poison: allocation" "$out.all" >> "$out"
grep "runs differ" "$out.all" >> "$out"
for ((i = 0; i < n && i < max; i++)); do
  timeout -k 10 120 env KSS_POISON=$i python -u tools/diag_flake.py single 1 > "$out.$i" 2>&1 || { echo "index $i: run failed" >> "$out"; exit 1; }
  echo "index $i: $(grep 'runs differ' "$out.$i")" >> "$out"
done
