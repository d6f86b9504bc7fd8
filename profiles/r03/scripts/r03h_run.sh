# round 3: N = 8 proxy: the display rank's shade on its own stream vs on the frame streams
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
for r in 1 2; do
  for v in ss base; do
    X=""; [ $v = ss ] && X="--shade-stream"
    timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 3 --shards 0,1 --windows 7 --sustain-steps 400 \
      --deal rr $X --cache /tmp/och_d12.npz --out $O/proxy_${v}_$r.json > $O/proxy_${v}_$r.log 2>&1 || exit 2
    echo "$v $r"; grep world $O/proxy_${v}_$r.log | grep -v summary | cut -c1-60,250-420
  done
done
