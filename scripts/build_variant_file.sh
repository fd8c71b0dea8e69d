#!/bin/bash
# Build a variant of libthesia with one source file compiled with extra -D flags (A/B only).
# Usage: scripts/build_variant_file.sh NAME csrc/FILE.hip "-DFLAG=..." -> lib/vd/NAME.so
set -e
cd "$(dirname "$0")/../multi-spectrogram-viewer_amd"
make -s -j8 >/dev/null
mkdir -p build/vd lib/vd
base=$(basename $2 .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -Wall -Wno-unused-function -fno-slp-vectorize $3 -c $2 -o build/vd/$1.o
objs=$(ls build/*.o | grep -v "/${VD_REPLACES:-$base}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/vd/$1.so $objs build/vd/$1.o -Wl,-rpath,/opt/rocm/lib
echo "lib/vd/$1.so"
