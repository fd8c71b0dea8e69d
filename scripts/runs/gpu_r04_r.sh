#!/bin/bash
# Round 4: PMC of the C5 display phase per step (all display kernels of one pass: HBM traffic and
# VALU instructions), scripts/c5_display_only.py 4 -> 5 display passes per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_r}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/scripts/c5_display_only.py 4 0"
timeout -k 10 200 python3 $B > $O/plain.txt 2>&1 || { tail $O/plain.txt; exit 1; }
cat $O/plain.txt
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "grey_vert|resize_h|render_stripe" -d $O/pmc_$i -o p --output-format csv -- python3 $B > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmc_$i.log; exit 1; }
  i=$((i+1))
done
python3 - $O 5 <<'PY'
import csv, glob, sys, collections
o, passes = sys.argv[1], int(sys.argv[2])
tot = collections.defaultdict(float)
per = collections.defaultdict(float)
for f in sorted(glob.glob(o + "/pmc_*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("thesia::", "").replace("(anonymous namespace)::", "")
        c = n.find(">(")
        n = n[:c + 1] if c >= 0 else n.split("(")[0]
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        per[(n.split("<")[0], r["Counter_Name"])] += float(r["Counter_Value"])
print("per display pass (sum over its launches):")
for k in sorted(tot):
    print(" ", k, "%.4g" % (tot[k] / passes))
print("per kernel family, per pass:")
for k in sorted(per):
    print(" ", k[0], k[1], "%.4g" % (per[k] / passes))
PY
echo done
