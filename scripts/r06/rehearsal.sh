#!/bin/bash
# 2-rank rehearsal on one GPU: the C4 and C5 lines (C5: the
# conforming kernel-7 path, its default since round 6) at --gpus 2 (two ranks
# share the device, as bench.py maps LOCAL_RANK % device_count), beside the N=1 lines of the
# same box, and the per-rank frame counts. The driver's 8-GPU run is not ours to launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06_rehearsal}
mkdir -p $O
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python bench.py --no-exact > $O/c4_n1.json 2> $O/c4_n1.err || { tail -5 $O/c4_n1.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --no-exact > $O/c4_n2.json 2> $O/c4_n2.err || { tail -5 $O/c4_n2.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 > $O/c5_n1.json 2> $O/c5_n1.err || { tail -5 $O/c5_n1.err; exit 1; }
timeout -k 10 300 python bench.py --workload c5 --gpus 2 > $O/c5_n2.json 2> $O/c5_n2.err || { tail -5 $O/c5_n2.err; exit 1; }
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for w in ("c4", "c5"):
    for n in (1, 2):
        d = json.loads(open(f"{o}/{w}_n{n}.json").read().strip().splitlines()[-1])
        c = d["config"]
        print(w, "N=%d" % n, "value %.4g" % d["value"], "ms/step %.3f" % d["ms_per_step"], "ranks", c.get("ranks"),
              "devices", c.get("devices"), "per_rank_frames", c.get("per_rank_frames"))
    # weak scaling: rank 0's shard at N=2 is the N=1 line's per-GPU workload
    f1 = json.loads(open(f"{o}/{w}_n1.json").read().strip().splitlines()[-1])["config"]["per_rank_frames"]
    f2 = json.loads(open(f"{o}/{w}_n2.json").read().strip().splitlines()[-1])["config"]["per_rank_frames"]
    print(w, "rank 0's shard at N=2 equals the N=1 line:", f2[0] == f1[0], f1[0], f2[0])
PY
