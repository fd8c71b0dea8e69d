#!/bin/bash
# Round 4: the changed GPU tests (C2 direct bounds, library pool, stripe display), the C5 line
# with render paths 0 (single-pass stripes) / 3 (two kernels for every group) A/B, a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_gpu_multitrack.py tests/test_gpu_napi.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
grep "C2 \|passed\|failed" $O/pytest.txt
cd /tmp
timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 --render-paths 0,3 --spec-policies 0,1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
grep render_paths $O/bench_c5.json
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline']['overlapped_ms'], d['roofline']['batches_policy_ms'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 > $O/kt.log 2>&1 || exit $?
python3 $R/scripts/kt_summary.py c5 $O/kt/kt_kernel_trace.csv > $O/kt_summary.txt || exit $?
cat $O/kt_summary.txt
echo done
# stft5 phase-ring variant (experiment library): parity, then an in-process A/B on C4
cd $R
EXP=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so
THESIA_LIB=$EXP timeout -k 10 200 python3 scripts/check_variant.py 1 > $O/variant1_parity.txt 2>&1; rc=$?
cat $O/variant1_parity.txt
if [ $rc -eq 0 ]; then
  THESIA_LIB=$EXP timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --variants 0,1 > $O/bench_c4_variants.json 2> $O/bench_c4_variants.err || exit $?
  grep variants_kernel_ms $O/bench_c4_variants.json
fi
echo done2
