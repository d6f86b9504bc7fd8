#!/bin/bash
# SQ instruction-mix and wait counters of the render kernel (one PMC pass,
# 8 SQ counters), for library variant $1 (build_variants name or "main").
set -o pipefail
V=${1:-main}; mkdir -p gpurun_out/pmc_$V
export TMPDIR=/tmp OCH_TREE_CACHE=/tmp/och_tree_d12.npz
[ "$V" != main ] && export OCH_GPU_LIB=build_variants/liboch_gpu_$V.so
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_$V -o run -- \
    python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-bounce > gpurun_out/pmc_$V/bench.json 2> gpurun_out/pmc_$V/err.log
