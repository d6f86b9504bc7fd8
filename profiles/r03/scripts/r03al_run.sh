# round 3: the driver's exact N = 1 command, five fresh processes (spread of the 20-step value)
set -o pipefail
O=gpurun_out/r03al; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
