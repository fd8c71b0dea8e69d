#!/bin/bash
# rocprofv3 evidence for the bench kernel: kernel-trace + stats, then one PMC pass per counter
# set (separate runs, never combined with tracing). Output under gpurun_out/prof_*.
#   BENCH_ARGS      bench.py args for the kernel-trace run
#   PMC_BENCH_ARGS  bench.py args for the PMC passes
#   PMC_SETS        ';'-separated counter sets (default: FETCH_SIZE; WRITE_SIZE; an SQ set)
set -u
REPO="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$REPO/gpurun_out"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BARGS=${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu-baseline}
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ "${SKIP_KT:-0}" != 1 ]; then
  rocprofv3 -L > "$OUT/rocprof_counters.txt" 2>&1 || true
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_kt" -o kt --output-format csv -- python3 "$REPO/bench.py" $BARGS > "$OUT/prof_kt.log" 2>&1
  rc=$?; echo "kt rc=$rc"; crash $rc && exit $rc
fi
PB=${PMC_BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-rfft-roofline}
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
IFS=';' read -ra sets <<< "$SETS"
for c in "${sets[@]}"; do
  tag=$(echo $c | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/prof_pmc_$tag" -o pmc --output-format csv -- python3 "$REPO/bench.py" $PB > "$OUT/prof_pmc_$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; crash $rc && exit $rc
done
exit 0
