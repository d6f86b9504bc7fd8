# round 3: N = 8 proxy (every shard) for two kernel libraries, interleaved
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
for r in 1 2; do
  for v in base asm; do
    OCH_GPU_LIB=build_variants/liboch_gpu_$v.so timeout -k 10 300 python -u tools/proxy_rank.py --worlds 8 --inflight 3 \
      --shards all --windows 5 --sustain-steps 300 --cache /tmp/och_d12.npz --out $O/proxy_${v}_$r.json > $O/proxy_${v}_$r.log 2>&1 || exit 1
    echo "$v $r $(grep summary $O/proxy_${v}_$r.log)"
  done
done
