# round 3: bench (tiled batch two views), proxy per world in fresh processes
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 2
for w in 8 4 2; do
  timeout -k 10 300 python -u tools/proxy_rank.py --worlds $w --inflight 3 --shards all --windows 5 --sustain-steps 300 \
     --cache /tmp/och_d12.npz --out $O/proxy_w$w.json >> $O/proxy.log 2>&1 || exit 5
done
timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 3 --shards all --windows 5 --sustain-steps 300 \
     --shade all --cache /tmp/och_d12.npz --out $O/proxy_w8_shadeall.json >> $O/proxy.log 2>&1 || exit 6
