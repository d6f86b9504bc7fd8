#!/bin/bash
# Run on the GPU box: rocprofv3 kernel trace + stats of bench.py, then
# separate PMC passes (never combined with tracing domains, per pool rules).
# Usage: bash tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python bench.py --steps 10 --warmup 3 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace_bench.json 2> $OUT/trace.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $BENCH > /dev/null 2> $OUT/pmc_fetch.err || exit 1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_tcc -o run -- $BENCH > /dev/null 2> $OUT/pmc_tcc.err || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- $BENCH > /dev/null 2> $OUT/pmc_sq.err || exit 1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d $OUT/pmc_misc -o run -- $BENCH > /dev/null 2> $OUT/pmc_misc.err || true
find $OUT -name '*.csv' | head -50
