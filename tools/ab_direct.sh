# A/B at N = 1: the fused launch writing RGBA8 frames (direct) vs codes + shade pass.
# Interleaved arms, fresh process each (stream-to-queue mapping).
set -o pipefail
O=${O:-gpurun_out/ab_direct}; mkdir -p $O
export OCH_TREE_CACHE=/tmp/och_tree_d12.npz
ARGS="--no-cpu-baseline --no-parity --no-other-configs --no-bounce --no-cull-off --sustain 1"
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py $ARGS > $O/direct_$r.json 2>> $O/err.log || exit 1
  timeout -k 10 200 python -u bench.py $ARGS --no-direct > $O/codes_$r.json 2>> $O/err.log || exit 2
done
python - <<'PY'
import json, glob, os
O = os.environ.get("O", "gpurun_out/ab_direct")
for arm in ("direct", "codes"):
    rows = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(f"{O}/{arm}_*.json"))]
    print(arm, [r["value"] for r in rows], [r["sustained"]["value"] for r in rows],
          [r["roofline"]["kernel_ms_serial"] for r in rows])
PY
