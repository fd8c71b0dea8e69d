#!/bin/bash
# C5 spectrogram phase: stft3 parity tests, the C5 bench line, one SQ pass over its stft3
# launches (LDS bank conflicts per n_fft instance).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r05_c5spec}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_streaming.py tests/test_gpu_viewer_geometry.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('C5', d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline']['overlapped_ms'])"
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES --kernel-include-regex "stft3" -d $O/pmc -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -3 $O/pmc.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(o + "/pmc/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
for k in sorted(tot):
    print(k[0], k[1], "%.4g" % (tot[k] / n[k]), n[k])
PY
