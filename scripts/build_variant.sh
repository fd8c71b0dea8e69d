#!/bin/bash
# Experiment helper: rebuild stft3_kernels.hip with extra compiler flags into a variant
# library lib/libthesia_<name>.so (the other objects are reused), for A/B runs with
# THESIA_LIB=.../lib/libthesia_<name>.so python bench.py ...
#   usage: scripts/build_variant.sh <name> <extra hipcc flags...>
set -eu
cd "$(dirname "$0")/../multi-spectrogram-viewer_amd"
name=$1; shift
FLAGS="-DTHESIA_EXPERIMENTS -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function"
mkdir -p build/var_$name lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS "$@" -c csrc/stft3_kernels.hip -o build/var_$name/stft3_kernels.o
objs=$(ls build/*.o | grep -v stft3_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libthesia_$name.so $objs build/var_$name/stft3_kernels.o -Wl,-rpath,/opt/rocm/lib
echo "built lib/libthesia_$name.so"
