# round 3: the default bench line with the moving-camera window
set -o pipefail
O=gpurun_out/r03ab; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
