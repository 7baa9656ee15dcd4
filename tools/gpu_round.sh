# parity tests, then phase stamps, then the C2 bench sweep
set -e
bash tools/gpu_simple.sh
bash tools/gpu_stamps2.sh
