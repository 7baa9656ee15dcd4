bash tools/ab_run.sh n2 base; bash tools/gpurecipe.sh n2 c4 c3
