# round 3: prepared N = 1 step issue vs the wrapper path; host timeline of the window
set -o pipefail
O=gpurun_out/r03v; mkdir -p $O
export TMPDIR=/tmp
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
B="--steps 20 --warmup 5 --extra-windows 3 --no-cpu-baseline --no-other-configs --no-bounce --sustain 0.5"
for m in fast slow fast slow; do
  X=""; [ $m = slow ] && X="--no-fast-issue"
  timeout -k 10 300 python -u bench.py $B $X > $O/b_$m.json 2> $O/b_$m.err || exit 2
  cp $O/b_$m.json $O/b_${m}_$(date +%s%N).json
done
EXTRA="$EXTRA" bash tools/r03t_run.sh || exit 3
cp gpurun_out/r03t/stamps.txt $O/stamps_fast.txt
