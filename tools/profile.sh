#!/bin/bash
# Run on the GPU box: rocprofv3 kernel trace of bench.py (timestamps only),
# then one separate PMC pass per counter group (never combined with tracing
# domains, per pool rules), then summarise the bench's headline window (the
# dispatches between its two marker kernels) into gpurun_out/prof_<tag>/:
#   summary.json        per-kernel PMC means (tools/pmc_summary.py --window)
#   window_summary.json the window's kernel timeline (tools/window_trace.py)
# Usage: bash tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r03}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export OCH_TREE_CACHE=${OCH_TREE_CACHE:-/tmp/och_tree_d12.npz}
BARGS="--steps 20 --no-cpu-baseline --no-parity --sustain 0 --no-other-configs --no-bounce --no-cull-off --no-split-arm $*"
step() {   # step <name> <rocprofv3 args...>
    local name=$1; shift
    echo "[profile] $name" >&2
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python -u bench.py $BARGS \
        > $OUT/$name.json 2> $OUT/$name.err
}
step trace --kernel-trace --stats || exit 1
step pmc_fetch --pmc FETCH_SIZE || exit 1
step pmc_write --pmc WRITE_SIZE || exit 1
step pmc_tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
step pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS || exit 1
step pmc_sq2 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY || exit 1
step pmc_sq3 --pmc SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
step pmc_grbm --pmc GRBM_GUI_ACTIVE || exit 1
python tools/pmc_summary.py $OUT --window --update $OUT/pmc_summary.json --key ${PMC_KEY:-d12_1920x1080_n1} \
    > $OUT/summary.json || exit 2
python tools/window_trace.py $OUT/trace --steps 20 --bench-json $OUT/trace.json --config ${PMC_KEY:-d12_1920x1080_n1} \
    --out $OUT/window_summary.json --csv $OUT/window_trace.csv > /dev/null || exit 3
# keep what is judged (summaries, kernel stats); the per-dispatch CSVs stay on the box
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
find $OUT -name "run_*.csv" -delete
