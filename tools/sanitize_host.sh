#!/bin/bash
# Host-code sanitizer run (CPU only; GPU sanitizers are not available on this
# pool): builds the oracle and the product library's host code with
# AddressSanitizer + UndefinedBehaviorSanitizer into a scratch directory (the
# device code object is the normal build's, untouched) and runs the CPU tests
# that exercise them -- the oracle's pins, cull, bounce, table and layout tests
# against the sanitized oracle; the builder, editor and ABI tests against the
# sanitized library.  Exit status: the tests'; any sanitizer report is printed.
# Usage: bash tools/sanitize_host.sh [scratch_dir]
set -o pipefail
cd "$(dirname "$0")/.."
S=${1:-/tmp/och_sanitize}
mkdir -p "$S"
make -s -C octree_ray_tracing_amd/csrc || exit 1
make -s -C oracle build/liboch_oracle.so || exit 1

# oracle: gcc's runtimes; swapped in for the run, restored after
gcc -std=c11 -O1 -g -march=x86-64-v3 -ffp-contract=off -fno-fast-math -fPIC -fno-omit-frame-pointer \
    -fsanitize=address,undefined -shared -pthread -o "$S/liboch_oracle.so" oracle/och_oracle.c -lm || exit 1
cp oracle/build/liboch_oracle.so "$S/liboch_oracle.so.orig"
cp "$S/liboch_oracle.so" oracle/build/liboch_oracle.so
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    timeout 1500 python -m pytest tests/test_oracle_pins.py tests/test_octree_table.py tests/test_cull.py \
    tests/test_bounce.py tests/test_packed_layout.py tests/test_palette.py -q -m "not gpu" 2>&1 | tee "$S/oracle.log"
rc1=$?
cp "$S/liboch_oracle.so.orig" oracle/build/liboch_oracle.so

# product library: host code with clang's runtimes (each -fsanitize= after -Xarch_host)
H=/opt/rocm/bin/hipcc
F="-std=c++17 -O1 -g -fPIC -ffp-contract=off -fno-fast-math -fno-omit-frame-pointer"
D="--offload-arch=gfx950 -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics"
X="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined"
C=octree_ray_tracing_amd/csrc
$H $F $D $X -msse2 -c $C/och_api.cpp -o "$S/och_api.o" &&
$H $F $D $X -c $C/och_builder.cpp -o "$S/och_builder.o" &&
$H $F $X -c $C/och_editor.cpp -o "$S/och_editor.o" &&
$H $F $X -c $C/och_group.cpp -o "$S/och_group.o" &&
$H $F $X -c $C/och_comm.cpp -o "$S/och_comm.o" &&
$H -shared -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -shared-libsan \
    -o "$S/liboch_gpu.so" $C/build/och_kernels.o "$S"/och_{api,builder,editor,group,comm}.o -pthread -ldl || exit 1
ASANRT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
OCH_GPU_LIB="$S/liboch_gpu.so" LD_PRELOAD="$ASANRT" ASAN_OPTIONS=detect_leaks=0 \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    timeout 1500 python -m pytest tests/test_builder.py tests/test_editor.py tests/test_abi.py -q -m "not gpu" \
    --deselect tests/test_abi.py::test_header_is_plain_c_and_links 2>&1 | tee "$S/library.log"
rc2=$?
grep -hE "runtime error|ERROR: AddressSanitizer" "$S/oracle.log" "$S/library.log" && exit 1
exit $(( rc1 || rc2 ))
