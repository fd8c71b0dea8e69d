set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "render or display or e2e or multitrack or exact or ragged" > gpurun_out/hseg_tests.log 2>&1
rc=$?; tail -3 gpurun_out/hseg_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/runs/gpu_vd_ab.sh
