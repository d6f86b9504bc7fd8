#!/bin/bash
# Heavy-tile split thresholds, interleaved: bench.py at N = 1 (its 20-step
# window, sustained and lone launch) and the N = 2 / 4 / 8 proxies
# (tools/proxy_rank.py, every shard, one fresh process per arm, bench.py's
# per-N frames in flight, queues and display weight).
# usage: bash tools/split_sweep.sh OUTDIR ROUNDS "T1 T2 ..." [WORLDS]   (T = 0: no split)
set -o pipefail
out=${1:?outdir}; rounds=${2:-2}; arms=${3:-"0 50"}; worlds=${4:-"1 8"}
mkdir -p "$out"
BA="--steps 20 --warmup 5 --no-other-configs --no-cpu-baseline --no-bounce --moving-steps 0 --no-cull-off"
for r in $(seq "$rounds"); do
  for t in $arms; do
    opt="--opt split=0"; [[ "$t" != 0 ]] && opt="--opt split=$t --opt split_segs=4 --opt split_level=6"
    for w in $worlds; do
      if [[ "$w" == 1 ]]; then
        timeout -k 10 200 python -u bench.py $BA $opt > "$out/n1_t${t}_r$r.json" 2> "$out/n1_t${t}_r$r.err" \
          || { tail -20 "$out/n1_t${t}_r$r.err"; exit 1; }
        echo "n1 T=$t r$r: $(python tools/bench_line.py "$out/n1_t${t}_r$r.json")"
      else
        q=""; f=3; dw=""
        [[ "$w" -ge 8 ]] && { q="GPU_MAX_HW_QUEUES=8"; f=6; }
        dw=$(python -c "import octree_ray_tracing_amd as o; print(o.display_weight($w, 'all_gather'))")
        env $q timeout -k 10 300 python -u tools/proxy_rank.py --worlds $w --inflight $f --shards all --events \
          --display-weight $dw $( [[ "$w" -ge 8 ]] && echo "--opt plan=0" ) $opt --out "$out/n${w}_t${t}_r$r.json" \
          > "$out/n${w}_t${t}_r$r.log" 2>&1 || { tail -20 "$out/n${w}_t${t}_r$r.log"; exit 2; }
        echo "n$w T=$t r$r: $(tail -1 "$out/n${w}_t${t}_r$r.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['slowest_ms_per_step_20'], d['slowest_ms_per_step_sustained'], d['job_mrays_s_20'], d['job_mrays_s_sustained'])")"
      fi
    done
  done
done
