set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "render or display or e2e or multitrack or exact or ragged" > gpurun_out/rp_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --render-paths 0,4 > gpurun_out/rp_ab.log 2>&1 || exit $?
grep render_paths gpurun_out/rp_ab.log
