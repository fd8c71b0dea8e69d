"""Multi-GPU sharding logic on CPU: the LPT partition and the one scalar
exchange of the display path (lib.rs:193-263), including a world_size-2 gloo run."""
import math
import os
import socket

import numpy as np
import pytest

import oracle_ffi as O
from thesia import shard


def test_lpt_partition_is_disjoint_complete_and_balanced():
    rng = np.random.default_rng(0)
    lens = rng.integers(48000, 48000 * 60, size=257)
    costs = [shard.track_cost(int(n), 2048, 512, 2048, 128) for n in lens]
    for ws in (1, 2, 3, 8):
        shards = shard.assign_tracks(costs, ws)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(costs)))
        loads = [sum(costs[i] for i in s) for s in shards]
        # LPT bound: max load <= mean + max single cost
        assert max(loads) <= sum(costs) / ws + max(costs) + 1e-6
        assert shards == shard.assign_tracks(costs, ws)  # deterministic on every rank


def test_equal_tracks_split_evenly():
    costs = [shard.track_cost(1_440_000, 2048, 512, 2048, 128)] * 8000
    shards = shard.assign_tracks(costs, 8)
    assert [len(s) for s in shards] == [1000] * 8


def test_empty_rank_range_and_single_process_exchange():
    assert shard.local_range([], []) == (-math.inf, math.inf)
    mx, mn, sr = shard.global_db_range(-3.0, -200.0, 48000)
    assert (mx, mn, sr) == (-3.0, -123.0, 48000)
    mx, mn, _ = shard.global_db_range(5.0, -20.0, 8000)  # lib.rs:208: max clamped to 0
    assert (mx, mn) == (0.0, -20.0)


def _tracks():
    rng = np.random.default_rng(42)
    out = []
    for i, sr in enumerate([8000, 16000, 22050, 24000, 44100, 48000, 16000, 8000]):
        n = int(sr * (0.1 + 0.05 * i))
        amp = 10.0 ** (-i / 4)
        out.append(((rng.standard_normal(n) * amp).astype(np.float32), sr))
    return out


def _spec_range(x, sr):
    from thesia.utils import track_params
    win, hop, n_fft = track_params(sr)
    w = (O.hann(win) / np.float32(n_fft)).astype(np.float32)
    db = O.amp_to_db_default(O.norm(O.perform_stft(x, win, hop, n_fft, window=w)))
    return float(db.max()), float(db.min())


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tracks = _tracks()
    mine = shard.plan_shards([len(x) for x, _ in tracks], 1024, 256, 1024, 0, world, rank)
    ranges = [_spec_range(*tracks[i]) for i in mine]
    lmx, lmn = shard.local_range([r[0] for r in ranges], [r[1] for r in ranges])
    lsr = max((tracks[i][1] for i in mine), default=0)
    q.put((rank, mine, shard.global_db_range(lmx, lmn, lsr)))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world_size_2_gloo_matches_single_process():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    shards = [r[1] for r in res]
    assert sorted(shards[0] + shards[1]) == list(range(8)) and not set(shards[0]) & set(shards[1])
    # every rank ends with the same global range, equal to one process over all tracks
    tracks = _tracks()
    ranges = [_spec_range(x, sr) for x, sr in tracks]
    ref = shard.global_db_range(max(r[0] for r in ranges), min(r[1] for r in ranges),
                                max(sr for _, sr in tracks))
    assert res[0][2] == res[1][2] == ref


def _sub_worker(rank, world, port, q):
    """3 ranks; a subgroup {0, 2} stands in for an RCCL group (its gloo shadow forced): every rank
    creates the shadows eagerly, then only the subgroup's members exchange their ranges."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub = dist.new_group(ranks=[0, 2], backend="gloo")
    shard.init_host_groups([sub], force=True)
    out = None
    if rank in (0, 2):
        out = shard.global_db_range(-10.0 * (rank + 1), -100.0 - rank, 8000 * (rank + 1), group=sub)
    dist.barrier()
    q.put((rank, out, sorted(shard._GLOO_SHADOW)))
    dist.destroy_process_group()


def test_subgroup_exchange_with_eager_shadow_groups():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sub_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = shard.global_db_range(-10.0, -102.0, 24000)  # max over {0, 2}, min over {0, 2}
    assert res[0][1] == res[2][1] == ref and res[1][1] is None
    assert all(r[2] == [(0, 1, 2), (0, 2)] for r in res)  # same shadows on every rank, keyed by ranks


def test_non_gloo_group_without_shadow_is_an_error():
    class FakeDist:  # an RCCL default group, no init_host_groups call
        def get_world_size(self):
            return 2

        def get_backend(self, group=None):
            return "nccl"

        def get_process_group_ranks(self, group):
            return [0, 1]
    import pytest as _pt
    with _pt.raises(RuntimeError, match="init_host_groups"):
        shard._host_group(FakeDist(), None)


def test_display_cost_grows_with_each_term():
    base = dict(n_samples=480000, sr=48000, win_length=2048, hop_length=512, n_fft=2048, max_sr=48000)
    c = shard.display_cost(**base)
    assert c > 0
    assert shard.display_cost(**{**base, "n_samples": 960000}) > 1.9 * c  # T and nwidth double
    assert shard.display_cost(**base, nheight=1000) > 1.3 * c              # the image rows
    assert shard.display_cost(**base, px_per_sec=400.0) > c                # more columns
    # a lower-rate track of the same length: grey image taller (up_ratio), fewer frames
    lo = shard.display_cost(**{**base, "sr": 8000, "n_samples": 80000})
    assert 0 < lo < c
    assert shard._lanczos3_taps(6891, 1000) == 43 and shard._lanczos3_taps(140, 500) == 7


def _mixed_workload(n=1000, seed=7):
    """Mixed durations (1-60 s), rates, n_fft and image heights (the display phase is 72 % of a
    C5 step)."""
    rng = np.random.default_rng(seed)
    rates = [8000, 16000, 22050, 24000, 44100, 48000]
    ffts = [256, 512, 1024, 2048]
    heights = [200, 500, 800]
    spec, disp = [], []
    for _ in range(n):
        sr = int(rng.choice(rates))
        nf = int(rng.choice(ffts))
        nh = int(rng.choice(heights))
        ns = int(sr * rng.uniform(1.0, 60.0))
        spec.append(shard.track_cost(ns, nf, nf // 4, nf))
        disp.append(shard.display_cost(ns, sr, nf, nf // 4, nf, 48000, 100.0, nh))
    return spec, disp


@pytest.mark.parametrize("ws", [2, 4, 8])
def test_two_phase_partition_balances_both_phases(ws):
    """Both phases' per-rank loads within 5 % of their mean on a mixed workload (a scalar-cost
    LPT balances only the sum, and a step pays the slowest rank of each phase)."""
    spec, disp = _mixed_workload()
    shards = shard.assign_tracks_2phase(spec, disp, ws)
    assert sorted(i for s in shards for i in s) == list(range(len(spec)))
    assert shards == shard.assign_tracks_2phase(spec, disp, ws)  # deterministic on every rank
    for costs in (spec, disp):
        loads = [sum(costs[i] for i in s) for s in shards]
        mean = sum(loads) / ws
        assert max(abs(l - mean) for l in loads) <= 0.05 * mean, (ws, loads)


def test_two_phase_beats_spectrogram_only_lpt_on_display():
    """The spectrogram-only cost model (round 3) leaves the display phase unbalanced on a workload
    whose image heights vary; the two-phase partition does not."""
    spec, disp = _mixed_workload(400, seed=3)
    def spread(shards, costs):
        loads = [sum(costs[i] for i in s) for s in shards]
        return max(loads) / (sum(loads) / len(loads)) - 1.0
    old = shard.assign_tracks(spec, 8)
    new = shard.assign_tracks_2phase(spec, disp, 8)
    assert spread(new, disp) < spread(old, disp)
    assert spread(new, disp) <= 0.05 and spread(new, spec) <= 0.05
