#!/bin/bash
# GPU validation run: smoke, pytest -m gpu, short bench (+ C5 bench). Stops at the first
# crash-class exit (fault/abort/segv/timeout); an ordinary test failure (rc 1) still lets the
# bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 ${SMOKE_T:-300} python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; crash $rc && exit $rc
timeout -k 10 ${TEST_T:-900} python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; crash $rc && exit $rc
timeout -k 10 ${BENCH_T:-600} python -u bench.py ${BENCH_ARGS:---steps 10 --warmup 2} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; crash $rc && exit $rc
if [ "${C5:-1}" = 1 ]; then
  timeout -k 10 ${BENCH_T:-600} python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1
  rc=$?; echo "bench c5 rc=$rc"; tail -3 gpurun_out/bench_c5.log
fi
exit $rc
