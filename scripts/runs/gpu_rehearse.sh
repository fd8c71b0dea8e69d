#!/bin/bash
# Multi-rank rehearsal on one GPU (both ranks share device 0): the bench's own launcher and the
# driver's torch.distributed.run form; then the C3 line. Output: gpurun_out/rehearse_*.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > gpurun_out/rehearse_launcher.log 2>&1 || exit $?
tail -1 gpurun_out/rehearse_launcher.log | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > gpurun_out/rehearse_torchrun.log 2>&1 || exit $?
grep '^{' gpurun_out/rehearse_torchrun.log | tail -1 | cut -c1-400
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e > gpurun_out/rehearse_c3.log 2>&1 || exit $?
grep '^{' gpurun_out/rehearse_c3.log | tail -1 | cut -c1-600
