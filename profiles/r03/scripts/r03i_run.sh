# round 3: N = 8 proxy, row deal by count with a lighter display rank
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
for w in 0.6 0.8 0.45; do
  timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 3 --shards all --windows 5 --sustain-steps 300 \
    --deal count --display-weight $w --cache /tmp/och_d12.npz --out $O/proxy_count_$w.json > $O/proxy_count_$w.log 2>&1 || exit 2
  echo "count $w $(grep summary $O/proxy_count_$w.log)"
  grep world $O/proxy_count_$w.log | grep -v summary | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(' ', d['shard'], d['rays_per_step_rank'], d['ms_per_step_20'], d['ms_per_step_sustained'])"
done
