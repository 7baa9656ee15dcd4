R=$(pwd)
for c in 3a027a6 cb6f667 9e06be7; do
  (cd bisect/$c && timeout -k 10 200 python -u bench.py --scenarios 512 --steps 3 --warmup 1 --no-cpu > $R/gpurun_out/bis_$c.json 2> $R/gpurun_out/bis_$c.err); echo "$c rc=$?"
done
timeout -k 10 200 python -u bench.py --scenarios 512 --steps 3 --warmup 1 --no-cpu > gpurun_out/bis_head.json 2> gpurun_out/bis_head.err; echo "head rc=$?"
