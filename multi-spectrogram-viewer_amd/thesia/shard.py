"""Multi-GPU sharding of the spectrogram path.

Files are independent through the whole spectrogram stage (lib.rs:112-136 runs per track), so
they shard across ranks (one process per GPU) with no collective on the data path. The only
cross-track coupling in the reference is the global dB range and the maximum sample rate that
`update_spec_greys` reduces before any grey image is built (lib.rs:193-263): three scalars per
rank, exchanged with one all_reduce between the spectrogram phase and the display phase.

This module is host logic only (no device calls), so it is covered on CPU by world_size-2 gloo
tests; on the GPU box the same calls run over RCCL ("nccl") or gloo.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

from .utils import stft_n_frames


def track_cost(n_samples: int, win_length: int, hop_length: int, n_fft: int, n_mels: int = 0) -> float:
    """Kernel cost model of one track: frames x (FFT work + per-bin work + mel work)."""
    T = stft_n_frames(n_samples, win_length, hop_length)
    F = n_fft // 2 + 1
    return float(T) * (n_fft * math.log2(max(n_fft, 2)) + 2.0 * F + 2.0 * n_mels)


def _lanczos3_taps(src: int, dst: int) -> int:
    """Most taps of one axis of image 0.23's Lanczos3 resample (src -> dst): 2*ceil(3*ratio)+1
    where it downsamples, 7 where it does not (display.rs:57; host_tables.cpp lanczos3_taps)."""
    if src <= 0 or dst <= 0:
        return 0
    ratio = max(src / dst, 1.0)
    return min(src, 2 * math.ceil(3.0 * ratio) + 1)


def display_cost(n_samples: int, sr: int, win_length: int, hop_length: int, n_fft: int, max_sr: int,
                 px_per_sec: float = 100.0, nheight: int = 500, n_mels: int = 0,
                 freq_scale_mel: bool = False) -> float:
    """Cost model of one track's display (grey + Lanczos3 + colormap, lib.rs:193-298 /
    display.rs:44-61), in HBM-byte equivalents: the dB rows read once (4*T*bins), the f32
    intermediate of the separable resize written and read ([nheight, T], 8*T*nheight), the RGB
    bytes written (3*nwidth*nheight), and the taps' arithmetic at the MI355X ridge of ~20 flop per
    byte (2 flop per tap: the vertical pass T*nheight*vtaps, the horizontal one
    nwidth*nheight*htaps). bins = n_mels or n_fft/2+1; H = round(bins*up_ratio)."""
    T = stft_n_frames(n_samples, win_length, hop_length)
    if T == 0 or nheight == 0:
        return 0.0
    bins = n_mels or n_fft // 2 + 1
    H = max(int(round(bins * up_ratio(sr, max_sr, freq_scale_mel))), bins)
    nwidth = int(px_per_sec * n_samples / sr)
    vt, ht = _lanczos3_taps(H, nheight), _lanczos3_taps(T, nwidth)
    bytes_ = 4.0 * T * bins + 8.0 * T * nheight + 3.0 * nwidth * nheight
    flops = 2.0 * (T * nheight * vt + nwidth * nheight * ht)
    return bytes_ + flops / 20.0


def assign_tracks(costs: Sequence[float], world_size: int) -> List[List[int]]:
    """Greedy LPT: tracks in decreasing cost (ties: lower index first) go to the least-loaded
    rank (ties: lower rank). Deterministic, so every rank computes the same partition without
    communicating. Returns, per rank, its track indices in increasing order."""
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    order = sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i))
    load = [0.0] * world_size
    shards: List[List[int]] = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += float(costs[i])
    return [sorted(s) for s in shards]


def assign_tracks_2phase(spec_costs: Sequence[float], disp_costs: Sequence[float],
                         world_size: int) -> List[List[int]]:
    """Greedy LPT over two phases that a step runs one after the other, with the range exchange
    between them (lib.rs:193-263: the display needs every rank's range first): a step takes the
    slowest rank's spectrogram phase plus the slowest rank's display phase, so each phase is
    balanced on its own. Each phase's costs are normalised by their total; tracks go in
    decreasing normalised sum (ties: lower index) to the rank whose larger normalised load after
    adding the track is smallest (ties: smaller sum, then lower rank). Deterministic on every
    rank. Returns, per rank, its track indices in increasing order."""
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    if len(spec_costs) != len(disp_costs):
        raise ValueError("one spectrogram and one display cost per track")
    A = float(sum(spec_costs)) or 1.0
    B = float(sum(disp_costs)) or 1.0
    a = [float(c) / A for c in spec_costs]
    b = [float(c) / B for c in disp_costs]
    order = sorted(range(len(a)), key=lambda i: (-(a[i] + b[i]), i))
    la = [0.0] * world_size
    lb = [0.0] * world_size
    shards: List[List[int]] = [[] for _ in range(world_size)]
    for i in order:
        r = min(range(world_size), key=lambda k: (max(la[k] + a[i], lb[k] + b[i]), la[k] + lb[k], k))
        shards[r].append(i)
        la[r] += a[i]
        lb[r] += b[i]
    return [sorted(s) for s in shards]


def local_range(spec_max: Sequence[float], spec_min: Sequence[float]) -> Tuple[float, float]:
    """Per-rank (max, min) over its tracks' dB spectrograms (lib.rs:194-207): -inf / +inf when the
    rank holds no track (ndarray-stats' EmptyInput -> unwrap_or)."""
    mx = max(spec_max, default=-math.inf)
    mn = min(spec_min, default=math.inf)
    return float(mx), float(mn)


def global_db_range(local_max: float, local_min: float, local_max_sr: int, db_range: float = 120.0,
                    group=None) -> Tuple[float, float, int]:
    """The display path's one exchange: global (max_db, min_db, max_sr) as lib.rs:194-228
    computes them over ALL tracks: max = min(max, 0), min = max(min, max - db_range).

    With torch.distributed initialised, reduces over `group` (default world) with one
    all_reduce(MAX) of (max, -min, max_sr) on host tensors; otherwise the local values are
    global. Three scalars are latency-bound on any transport, and the engine's buffers are not
    torch tensors, so a non-gloo group (RCCL "nccl") is shadowed by a gloo group over the same
    ranks (made once on every rank by init_host_groups) instead of staging the scalars on a GPU."""
    import numpy as np

    mx, mn, sr = float(local_max), float(local_min), int(local_max_sr)
    try:
        import torch
        import torch.distributed as dist
        active = dist.is_available() and dist.is_initialized()
    except ImportError:  # pragma: no cover - torch is in the image
        active = False
    if active and dist.get_world_size(group) > 1:
        g = _host_group(dist, group)
        t = torch.tensor([mx, -mn, float(sr)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
        mx, mn, sr = float(t[0]), -float(t[1]), int(t[2])
    # lib.rs:208-209 in f32, as the reference stores them
    gmax = float(np.float32(min(mx, 0.0)))
    gmin = float(np.float32(max(mn, gmax - db_range)))
    return gmax, gmin, sr


_GLOO_SHADOW = {}  # tuple of global ranks -> gloo group over them


def _ranks_key(dist, group):
    return tuple(range(dist.get_world_size())) if group is None else tuple(dist.get_process_group_ranks(group))


def init_host_groups(groups=(), force: bool = False) -> None:
    """Create the gloo groups the range exchange runs on: one over the world and one over each
    group in `groups`, in that order. Call it on EVERY rank, right after init_process_group:
    new_group is collective over the whole default group (ranks outside a subgroup must enter it
    too, in the same order), so creating a shadow lazily inside global_db_range -- where only a
    subgroup's members would call -- could deadlock or mismatch groups. With a gloo default group
    nothing is created (the groups themselves serve) unless `force` (tests: a gloo group standing
    in for an RCCL one)."""
    import torch.distributed as dist

    for g in (None,) + tuple(groups):
        if not force and dist.get_backend(g) == "gloo":
            continue
        key = _ranks_key(dist, g)
        if key not in _GLOO_SHADOW:
            _GLOO_SHADOW[key] = dist.new_group(ranks=list(key), backend="gloo")


def _host_group(dist, group):
    """The gloo group the three scalars are reduced on: a shadow made by init_host_groups for
    `group`'s ranks (keyed by the rank tuple, never by id(): a collected group's id can be
    reused), else `group` itself when it is gloo. A non-gloo group without a shadow is an error:
    a lazy new_group here could deadlock (see init_host_groups)."""
    key = _ranks_key(dist, group)
    if key in _GLOO_SHADOW:
        return _GLOO_SHADOW[key]
    if dist.get_backend(group) == "gloo":
        return group
    raise RuntimeError("global_db_range over a non-gloo group needs thesia.shard.init_host_groups() "
                       "called on every rank right after init_process_group")


def up_ratio(sr: int, max_sr: int, freq_scale_mel: bool) -> float:
    """Per-track vertical ratio of the grey image (lib.rs:231-248), in f32 like the reference."""
    import numpy as np
    from .mel import hz_to_mel

    if freq_scale_mel:
        return float(np.float32(hz_to_mel(max_sr / 2.0)) / np.float32(hz_to_mel(sr / 2.0)))
    return float(np.float32(max_sr) / np.float32(sr))


def plan_shards(n_samples: Sequence[int], win_length: int, hop_length: int, n_fft: int,
                n_mels: int, world_size: int, rank: Optional[int] = None):
    """Convenience: LPT partition of tracks with the given lengths; returns all shards, or
    rank's shard when `rank` is given."""
    costs = [track_cost(n, win_length, hop_length, n_fft, n_mels) for n in n_samples]
    shards = assign_tracks(costs, world_size)
    return shards if rank is None else shards[rank]
