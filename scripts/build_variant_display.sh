#!/bin/bash
# Build a variant of libthesia whose display_kernels.hip is compiled with extra -D flags (A/B of
# display compile-time choices; never the product library). Usage:
#   scripts/build_variant_display.sh NAME "-DTHESIA_VDEPTH=16 ..." -> multi-spectrogram-viewer_amd/lib/vd/NAME.so
set -e
cd "$(dirname "$0")/../multi-spectrogram-viewer_amd"
make -s -j8 >/dev/null
mkdir -p build/vd lib/vd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -Wall -Wno-unused-function -fno-slp-vectorize $2 -c csrc/display_kernels.hip -o build/vd/$1.o
objs=$(ls build/*.o | grep -v display_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/vd/$1.so $objs build/vd/$1.o -Wl,-rpath,/opt/rocm/lib
echo "lib/vd/$1.so"
