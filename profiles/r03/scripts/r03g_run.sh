# round 3: row-deal parity, then the N = 8 proxy with the cost deal vs round-robin
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_frame_group.py \
   tests/test_examples.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for d in cost rr; do
    timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 3 --shards all --windows 5 --sustain-steps 300 \
      --deal $d --cache /tmp/och_d12.npz --out $O/proxy_${d}_$r.json > $O/proxy_${d}_$r.log 2>&1 || exit 2
    echo "$d $r $(grep summary $O/proxy_${d}_$r.log)"
  done
done
