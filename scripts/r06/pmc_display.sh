#!/bin/bash
# SQ counters of the C5 display kernels (render path 0: the stripe kernel for the groups with >= 3
# frames per column, grey_vert + resize_h_dma for the others): LDS conflicts vs LDS / VALU work.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r06_pmc_display}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "render_stripe|grey_vert|resize_h" -d $O/pmc_$i -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline --no-exact > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmc_$i.log; exit 1; }
  i=$((i+1))
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in sorted(glob.glob(o + "/pmc_*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        nm = r["Kernel_Name"].split("(")[0]
        k = (nm[-60:], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
for k in sorted(tot):
    print(k[0], k[1], "%.4g" % (tot[k] / n[k]), "per launch over", n[k])
PY
