#!/bin/bash
# counters of one display group's kernels: gpu_r04_m.sh OUT GROUP PATH REGEX
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_m}
G=${2:-6}; P=${3:-0}; RX=${4:-resize_h}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/scripts/display_one_group.py $G $P 3"
timeout -k 10 120 python3 $B > $O/plain.txt 2>&1 || exit $?
cat $O/plain.txt
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
         "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_BUSY_avr" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex "$RX" -d $O/pmc_$i -o p --output-format csv -- python3 $B > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmc_$i.log; exit 1; }
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
    print(k[0], k[1], "%.4g" % (tot[k] / n[k]))
PY
echo done
