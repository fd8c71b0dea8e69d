#!/bin/bash
# Round 4: the device-side range path -- render/C5 parity tests (incl. the device-range test), the
# C5 line twice and the phase gap in a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "render or c5 or device_range" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_c5_$r.json 2> $O/bench_c5_$r.err || { tail -20 $O/bench_c5_$r.err; exit 1; }
tail -1 $O/bench_c5_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline']['overlapped_ms'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 5 --warmup 1 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 $R/scripts/kt_gaps.py $O/kt/kt_kernel_trace.csv
echo done
