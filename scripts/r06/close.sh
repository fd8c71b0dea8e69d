#!/bin/bash
# Round 6 close: the full GPU suite and smoke on the product library, the default bench line (C4)
# with its rocprofv3 kernel trace and PMC passes (FETCH / WRITE / SQ) of the stft5 launches, the
# C5 line with its kernel trace, the viewer line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r06_close}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -10 $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('roofline_valu_issue',{}).get('frac'))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
grep -i "stft5\|stftr" $O/kt/kt_kernel_stats.csv | cut -c1-200
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "stft5|stftr" -d $O/pmc_$i -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmc_$i.log; exit 1; }
  i=$((i+1))
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in sorted(glob.glob(o + "/pmc_*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
for k in sorted(tot):
    print(k[0], k[1], "%.4g" % (tot[k] / n[k]), "per launch over", n[k])
PY
cd $R
timeout -k 10 300 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; t=d['tolerance_path']; print('C5 (kernel 7)', d['ms_per_step'], d['roofline_display']['display_ms'], r['overlapped_ms'], 'tolerance', t['ms_per_step'], t['spectrogram_overlapped_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o kt --output-format csv -- python3 $R/bench.py --workload c5 --no-cpu-baseline > $O/kt_c5.log 2>&1 || { tail -5 $O/kt_c5.log; exit 1; }
cd $R
timeout -k 10 300 python bench.py --workload viewer > $O/bench_viewer.json 2> $O/bench_viewer.err || { tail -20 $O/bench_viewer.err; exit 1; }
tail -1 $O/bench_viewer.json | cut -c1-300
echo done
