#!/bin/bash
# Build an A/B measurement variant of libws_hip.so with extra -D flags on one kernel file
# (default ws_fused_dppy_f64_2.hip = the fp64 two-step dppy / x2y instantiations; e.g.
# the knobs in csrc/ws_knobs.h):
#   tools/variant.sh NAME "-DWS_DPPY_PF=3 ..." [file]  -> nvidia-jetson-workload_amd/lib/variants/libws_hip_NAME.so
set -eu
cd "$(dirname "$0")/../nvidia-jetson-workload_amd/csrc"
make -s -j8 >/dev/null
NAME=$1; DEFS=${2:-}; SRCS=${3:-ws_fused_dppy_f64_2.hip}  # one or more sources, space separated
mkdir -p _obj/var ../lib/variants
FLAGS="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -I/opt/rocm/include"
OBJS=$(ls _obj/*.hip.o _obj/*.cpp.o)  # (not -save-temps' per-target intermediates)
VOBJS=""
for SRC in $SRCS; do
  /opt/rocm/bin/hipcc $FLAGS $DEFS -c $SRC -o _obj/var/${NAME}_$SRC.o
  OBJS=$(echo "$OBJS" | grep -v "/${SRC}.o$")
  VOBJS="$VOBJS _obj/var/${NAME}_$SRC.o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/variants/libws_hip_$NAME.so $OBJS $VOBJS \
    -L/opt/rocm/lib -lrccl -lhipfft -Wl,-rpath,/opt/rocm/lib
echo "built lib/variants/libws_hip_$NAME.so"
