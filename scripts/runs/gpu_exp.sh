#!/bin/bash
# Ad-hoc GPU experiment: parity tests, then bench lines for the variants given in $BENCHES
# (';'-separated "ENV=.. args" specs). Stops at the first crash-class exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_T:-400} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; crash $rc && exit $rc
fi
i=0
IFS=';' read -ra specs <<< "${BENCHES:-}"
for spec in "${specs[@]}"; do
  i=$((i+1))
  echo "== bench $i: $spec"
  timeout -k 10 300 env $spec > gpurun_out/bench_$i.log 2>&1
  rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/bench_$i.log | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if 'value' in d: print('value %.4g ms %.3f kernel_ms %.3f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))
    else: print(l.strip())"; crash $rc && exit $rc
done
exit 0
