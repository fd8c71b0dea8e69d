#!/bin/bash
# Build a variant of libthesia whose stft5_kernels.hip is compiled with extra -D flags (A/B of
# stft5 compile-time choices; never the product library). Usage:
#   scripts/build_v5.sh NAME "-DTHESIA_SC5=0 ..."   ->  multi-spectrogram-viewer_amd/lib/v5/NAME.so
set -e
cd "$(dirname "$0")/../multi-spectrogram-viewer_amd"
make -s -j8 >/dev/null
mkdir -p build/v5 lib/v5
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -Wall -Wno-unused-function -fno-slp-vectorize $2 -c csrc/stft5_kernels.hip -o build/v5/$1.o
objs=$(ls build/*.o | grep -v stft5_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/v5/$1.so $objs build/v5/$1.o -Wl,-rpath,/opt/rocm/lib
echo "lib/v5/$1.so"
