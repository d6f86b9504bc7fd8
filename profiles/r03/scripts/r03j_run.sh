# round 3: N = 2 / 4 proxy, row deal by count with a lighter display rank
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
for wl in "4 1.0" "4 0.85" "4 0.7" "2 1.0" "2 0.9" "2 0.8"; do
  set -- $wl
  timeout -k 10 300 python -u tools/proxy_rank.py --worlds $1 --inflight 3 --shards all --windows 5 --sustain-steps 200 \
    --deal count --display-weight $2 --cache /tmp/och_d12.npz --out $O/proxy_w$1_$2.json > $O/proxy_w$1_$2.log 2>&1 || exit 2
  echo "N=$1 w=$2 $(grep summary $O/proxy_w$1_$2.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["slowest_ms_per_step_20"], d["job_mrays_s_20"], d["slowest_ms_per_step_sustained"], d["job_mrays_s_sustained"])')"
  grep world $O/proxy_w$1_$2.log | grep -v summary | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(' ', d['shard'], d['rays_per_step_rank'], d['ms_per_step_20'], d['ms_per_step_sustained'])"
done
