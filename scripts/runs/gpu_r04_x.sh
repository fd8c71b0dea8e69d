#!/bin/bash
# Round 4: stft5 at the 48 kHz viewer geometry -- viewer / mel / exactness tests, then the viewer
# bench lines with stft3 vs stft5 (mel-128 dB and amp dB, stereo 30 s x 1000), and the default C4 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_x}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_viewer_geometry.py tests/test_gpu_mel.py tests/test_gpu_stft.py tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for out in mel_db amp_db; do
  timeout -k 10 300 python bench.py --win 1920 --hop 480 --n-fft 2048 --output $out --kernels 3,5 --steps 10 --warmup 2 > $O/bench_view_$out.json 2> $O/bench_view_$out.err || { tail -20 $O/bench_view_$out.err; exit 1; }
  grep kernels_ms $O/bench_view_$out.json | cut -c1-300
  tail -1 $O/bench_view_$out.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$out', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo done
