#!/bin/bash
# counters of the stripe kernel on one group (44.1 kHz / 256: generator slot 4)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_f}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/scripts/display_one_group.py 4 0 3"
timeout -k 10 120 python3 $B > $O/plain.txt 2>&1 || exit $?
cat $O/plain.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B > $O/kt.log 2>&1 || exit $?
python3 $R/scripts/kt_summary.py g4 $O/kt/kt_kernel_trace.csv
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
         "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM_NORM GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "stripe" -d $O/pmc_$i -o p --output-format csv -- python3 $B > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmc_$i.log; exit 1; }
  i=$((i+1))
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in sorted(glob.glob(o + "/pmc_*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(k, tot[k] / n[k])
PY
echo done
