T=$1
bash tools/ab_run.sh $T base
bash tools/gpurecipe.sh $T tests
