# round 3: asm-load variant -- parity (full GPU suite on the variant lib), then interleaved A/B
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
OCH_GPU_LIB=build_variants/liboch_gpu_asm.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/tests_asm.log 2>&1 || exit 1
bash tools/ab_libs.sh asmload base asm > $O/ab.txt 2>&1 || exit 2
mv gpurun_out/ab_asmload_* $O/ 2>/dev/null
true
