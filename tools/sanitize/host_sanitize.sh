#!/bin/bash
# ASan + UBSan build of libws_hip.so's HOST code (the device code is unchanged: GPU
# sanitizers are not used) and a run of abi_host_check.c against it, on a GPU-less host.
# Needs the normal build's device objects (make -C nvidia-jetson-workload_amd/csrc).
set -eu
cd "$(dirname "$0")/../../nvidia-jetson-workload_amd/csrc"
OUT=${OUT:-/tmp/ws_host_sanitize}
mkdir -p "$OUT"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result -I../../include -I/opt/rocm/include"
for f in ws_runtime.cpp ws_schedule.cpp ws_autotune.cpp ws_slab.cpp ws_initial_conditions.cpp ws_comm.cpp; do
  /opt/rocm/bin/hipcc $FLAGS $SAN -x hip -c $f -o "$OUT/$f.o" &
done
wait
HIPOBJ=$(ls _obj/*.hip.o)
CLANG=/opt/rocm/lib/llvm/bin/clang
# Host-only link with plain clang++ (the device code objects are already embedded in the
# .o files): the sanitizer runtime is a host library, nothing here targets the GPU.
${CLANG}++ -shared -shared-libasan -fsanitize=address,undefined -o "$OUT/libws_hip_san.so" \
    "$OUT"/*.cpp.o $HIPOBJ -L/opt/rocm/lib -lamdhip64 -lrccl -lhipfft -Wl,-rpath,/opt/rocm/lib
$CLANG -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=all -shared-libasan -I../../include \
    ../../tools/sanitize/abi_host_check.c -o "$OUT/abi_host_check" -L"$OUT" -lws_hip_san -Wl,-rpath,"$OUT" \
    -Wl,-rpath,$(dirname $($CLANG -print-file-name=libclang_rt.asan-x86_64.so))
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/abi_host_check"
