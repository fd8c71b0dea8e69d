#!/bin/bash
# Round 6: HBM-side traffic of the C5 display phase (render path 0), re-measured on the round's
# library: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over scripts/c5_display_only.py
# 4 0 (5 display passes), summed over the display kernels' launches, per pass; KiB x 1024, FETCH
# x 2 (MI355X_MICROARCH.md's gfx950 correction).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r06_display_traffic}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "render_stripe|grey_vert|resize_h|range_global" -d $O/pmc_$i -o p --output-format csv -- python3 $R/scripts/c5_display_only.py 4 0 > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/pmc_$i.log; exit 1; }
  i=$((i+1))
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float)
fam = collections.defaultdict(float)
for f in sorted(glob.glob(o + "/pmc_*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        c = r["Counter_Name"]
        v = float(r["Counter_Value"])
        tot[c] += v
        nm = r["Kernel_Name"]
        k = "render_stripe" if "render_stripe" in nm else "grey_vert" if "grey_vert" in nm else "resize_h" if "resize_h" in nm else "other"
        fam[(k, c)] += v
passes = 5
fetch = tot["FETCH_SIZE"] / passes * 1024 * 2
write = tot["WRITE_SIZE"] / passes * 1024
print("per display pass: FETCH %.4g B (x2 applied)  WRITE %.4g B  total %.4g B" % (fetch, write, fetch + write))
for c in ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
    print("per display pass: %s %.4g" % (c, tot[c] / passes))
for (k, c), v in sorted(fam.items()):
    scale = 2048 if c == "FETCH_SIZE" else 1024 if c == "WRITE_SIZE" else 1
    print("  %s %s %.4g" % (k, c, v / passes * scale))
PY
