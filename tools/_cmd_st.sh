T=$1
bash tools/ab_run.sh $T base || exit 1
timeout -k 10 300 python -u tools/c2_stamps.py 2 0 32 48 64 80 > gpurun_out/${T}_stamps.txt 2>&1; echo "stamps rc=$?"; cat gpurun_out/${T}_stamps.txt | grep -v "^$" | head -60
