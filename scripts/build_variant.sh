#!/bin/bash
# Build a variant of libthesia with some sources recompiled under extra -D flags (A/B of
# compile-time choices; never the product library). Usage:
#   scripts/build_variant.sh NAME "-DTHESIA_V_ILP=0 ..." "display_kernels.hip engine.cpp"
#     ->  multi-spectrogram-viewer_amd/lib/var/NAME.so
set -e
cd "$(dirname "$0")/../multi-spectrogram-viewer_amd"
make -s -j8 >/dev/null
rm -rf build/var/$1; mkdir -p build/var/$1 lib/var
objs=""
for o in build/*.o; do
  b=$(basename $o .o); keep=1
  for src in $3; do [ "${src%.*}" = "$b" ] && keep=0; done
  [ $keep = 1 ] && objs="$objs $o"
done
for src in $3; do
  arch=""; [ "${src##*.}" = "hip" ] && arch="--offload-arch=gfx950 -fno-slp-vectorize"
  /opt/rocm/bin/hipcc $arch -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall \
    -Wno-unused-function $2 -c csrc/$src -o build/var/$1/${src%.*}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/var/$1.so $objs build/var/$1/*.o -Wl,-rpath,/opt/rocm/lib
echo "lib/var/$1.so"
