#!/bin/bash
# viewer-geometry streaming kernel: its tests, the GPU suite, and kernel A/B (stft2 vs stft3v)
# at the viewer geometries on C4-sized batches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-s2_view}; mkdir -p $O
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_viewer_geometry.py -q -x --timeout 240 --timeout-method thread > $O/pytest_view.txt 2>&1; rc=$?
[ "${SKIP_TESTS:-0}" = 1 ] || { tail -5 $O/pytest_view.txt; [ $rc -eq 0 ] || exit $rc; }
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
[ "${SKIP_TESTS:-0}" = 1 ] || { tail -2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc; }
NB="--no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline --steps 5 --warmup 2"
for cfg in ${CFGS:-} "--sr 48000 --n-fft 2048 --win 1920 --hop 480 --output mel_db" "--sr 48000 --n-fft 2048 --win 1920 --hop 480 --output amp_db" "--sr 24000 --n-fft 1024 --win 960 --hop 240 --output amp_db --seconds 60" "--sr 8000 --n-fft 512 --win 320 --hop 80 --output amp_db --seconds 180 --channels 1" "--sr 44100 --n-fft 2048 --win 1764 --hop 441 --output mel_db" "--sr 44100 --n-fft 2048 --win 1764 --hop 441 --output amp_db" "--sr 22050 --n-fft 1024 --win 884 --hop 221 --output amp_db --seconds 60" "--sr 44100 --n-fft 2048 --win 1764 --hop 441 --output amp_db --channels 1"; do
  timeout -k 10 300 python -u bench.py $cfg --kernels 2,3 $NB > $O/ab.log 2>&1 || exit $?
  echo "$cfg: $(grep kernels_ms $O/ab.log)"
done
