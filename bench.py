"""bench.py -- STFT frames/s of the MI355X engine on BASELINE.json's multi-GPU workload.

Workload ("C4 per-GPU shard", BASELINE.json configs[3]): every rank owns 1000 synthetic
48 kHz 30 s stereo tracks (int16-quantised chirp + noise, stored as interleaved f32 -- the
reference's in-memory format after open_audio_file, audio.rs:9-37), resident in HBM before
timing. One step = one pass of the hot path over the rank's whole shard: channel-sum
downmix (lib.rs:42) -> reflect framing + Hann/n_fft (lib.rs:367-440) -> real FFT
(realfft.rs) -> |X| (lib.rs:124) -> 128-band mel projection (lib.rs:131) -> amp dB
(decibel.rs:79-88), n_fft 2048 / hop 512 / win 2048, one launch of the streaming kernel
(stft3_kernel). Files shard across ranks by LPT (thesia.shard) with no
data-path collective ("weak" scaling: per-GPU work is fixed).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU; gloo is used only for the timing barrier / max).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))

import numpy as np  # noqa: E402

import thesia  # noqa: E402  (loads libthesia before torch: one HIP runtime in the process)
from thesia import engine, shard  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", choices=["c4", "c3", "c5"], default="c4",
                   help="c4 (default, BASELINE.json metric): 48 kHz 30 s stereo, mel-128; "
                        "c3: 48 kHz 10 s mono, mel-128; c5: mixed rates / n_fft, dB + RGB render")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--tracks", type=int, default=1000, help="tracks per GPU")
    p.add_argument("--seconds", type=float, default=None, help="default 30 (c4) / 10 (c3, c5)")
    p.add_argument("--sr", type=int, default=48000)
    p.add_argument("--channels", type=int, default=None, help="default 2 (c4) / 1 (c3, c5)")
    p.add_argument("--input", choices=["f32", "s16"], default="f32")
    p.add_argument("--n-fft", type=int, default=2048)
    p.add_argument("--hop", type=int, default=512)
    p.add_argument("--n-mels", type=int, default=128)
    p.add_argument("--output", choices=["mel_db", "amp_db", "power_db", "complex"], default="mel_db")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-rfft-roofline", action="store_true",
                   help="skip the extra complex-output (window+rFFT kernel) roofline measurement")
    p.add_argument("--cpu-workers", type=int, default=16)
    p.add_argument("--variants", default="", help="experiment: comma list of THESIA_STFT_VARIANT "
                   "values to A/B (interleaved rounds, one process); prints per-variant kernel ms")
    a = p.parse_args()
    if a.seconds is None:
        a.seconds = 30.0 if a.workload == "c4" else 10.0
    if a.channels is None:
        a.channels = 2 if a.workload == "c4" else 1
    return a


def dist_setup(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        pg = dist
    return ws, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def max_over_ranks(pg, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def algorithmic_bytes(args, n_tracks, n_samples, total_frames, row_bins):
    """Bytes one launch must move at least: the input once (hop-strided, not n_fft per frame)
    plus the output rows (DESIGN.md §4 'Roofline and algorithmic bytes')."""
    in_el = 4 if args.input == "f32" else 2
    out_el = 8 if args.output == "complex" else 4
    return n_tracks * n_samples * args.channels * in_el + total_frames * row_bins * out_el


def cpu_baseline(args, n_samples):
    """The oracle (oracle/thesia_oracle.c, a C restatement of the reference path) on a
    bounded sample of the same workload: per-track parallel with one plan per track, like
    the reference's rayon path (lib.rs:161-166)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    from concurrent.futures import ThreadPoolExecutor

    workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
    n_tracks = 3 * workers  # ~10-15 s of CPU work on 16 threads
    fb = O.calc_mel_fb(args.sr, args.n_fft, args.n_mels)
    pcm = [engine.synth_pcm_host(args.channels, i, n_samples, args.sr).astype(np.float32) / 32768.0
           for i in range(n_tracks)]

    def one(x):
        mono = np.zeros(x.shape[0], np.float32)
        for c in range(x.shape[1]):
            mono = (mono + x[:, c]).astype(np.float32)
        X = O.perform_stft(mono, args.n_fft, args.hop, args.n_fft)
        db = O.amp_to_db_default(O.dot(O.norm(X), fb))
        return db.shape[0]

    t0 = time.perf_counter()
    with ThreadPoolExecutor(workers) as ex:
        frames = sum(ex.map(one, pcm))
    dt = time.perf_counter() - t0
    return {"value": frames / dt, "unit": "frames/s", "cores": workers, "kind": "port",
            "sample": f"{n_tracks} tracks x {args.seconds:g} s x {args.channels} ch @ {args.sr} Hz "
                      f"({frames} frames, {dt:.2f} s wall) through the C oracle, {workers} threads"}


def rfft_roofline(args, din, offs, lens, fmt, n_local, n_samples):
    """BASELINE.json north_star's "window+rFFT kernel" on the same resident input: the same
    streaming kernel with complex-spectrum output ([T, F] complex64, perform_stft's result,
    lib.rs:436-440), timed with HIP events on its launch stream; algorithmic bytes = input once
    + F x 8 B per frame. Reported beside the headline roofline, never as `value`."""
    plan = engine.Plan(args.n_fft, args.n_fft, args.hop, engine.OUT_COMPLEX, sr=args.sr)
    frames = engine.Batch.frames_for(plan, lens)
    dout = engine.DeviceBuffer(frames * plan.row_bins * 8)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=args.channels)
    b.run_timed(2)
    kms = b.run_timed(5) / 5
    in_el = 4 if args.input == "f32" else 2
    abytes = n_local * n_samples * args.channels * in_el + frames * plan.row_bins * 8
    achieved = abytes / (kms * 1e-3) / 1e9
    b.close()
    dout.close()
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "kernel_ms": kms, "algorithmic_bytes_per_launch": abytes,
            "frames_per_s": frames / (kms * 1e-3),
            "kernel": "thesia::stft3_kernel, complex output (downmix+frame+window+rFFT)"}


def frames_all_ranks(pg, frames: int) -> int:
    if pg is None:
        return frames
    import torch
    t = torch.tensor([float(frames)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return int(t.item())


def traffic_from_profile(workload_key):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        rec = d.get(workload_key)
        return None if rec is None else rec.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main_c5(args, ws, rank, pg):
    """C5 (BASELINE.json configs[4]): mixed-rate tracks with per-track n_fft, amp dB, global
    range exchange, grey + Lanczos3 + colormap RGB for every track (thesia.pipeline). One step =
    spectrogram launches for every geometry group + the display path of every track, the RGB
    images left in HBM (the copy to the host that get_spec_image implies, lib.rs:294-298, is
    timed separately: PCIe-inclusive, never the reported value)."""
    from thesia import pipeline

    total = args.tracks * ws
    gen = pipeline.c5_tracks(total, seconds=0.0)  # geometry only (empty PCM) for the partition
    costs = [shard.track_cost(int(round(args.seconds * t.sr)), t.n_fft, t.n_fft // 4, t.n_fft)
             for t in gen]
    mine = shard.assign_tracks(costs, ws)[rank]
    tracks = []
    for i in mine:  # the generator is indexed by the global track id
        tracks += pipeline.c5_tracks(1, seconds=args.seconds, first=i, channels=args.channels)
    p = pipeline.RenderPipeline(tracks, px_per_sec=100.0, nheight=500, pinned_output=True)

    def step(want_rgb=False):
        # images stay in HBM in the timed step (inputs resident, outputs resident); the
        # host-copy-inclusive rate is measured separately below
        p.run_spectrograms()
        p.render(group=None, want_rgb=want_rgb)

    for _ in range(args.warmup):
        step()
    engine.synchronize()
    barrier(pg)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    engine.synchronize()
    barrier(pg)
    dt = max_over_ranks(pg, (time.perf_counter() - t0) / args.steps)
    step(want_rgb=True)  # untimed: pins the host readback buffers once (hipHostRegister)
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step(want_rgb=True)
    engine.synchronize()
    dt_host = max_over_ranks(pg, (time.perf_counter() - t0) / 3)
    # spectrogram kernels alone (HIP events per group launch)
    kms = sum(b.run_timed(3) / 3 for _, _, _, b in p.groups)
    in_bytes = sum(t.pcm.nbytes for t in tracks)
    out_bytes = sum(b.total_frames * pl.row_bins * 4 for pl, _, _, b in p.groups)
    achieved = (in_bytes + out_bytes) / (kms * 1e-3) / 1e9
    frames_all = frames_all_ranks(pg, p.total_frames)
    if rank == 0:
        print(json.dumps({
            "metric": "STFT frames/sec (n_fft=2048 hop=512) at 1/2/4/8 GPUs; % HBM roofline",
            "value": frames_all / dt, "unit": "frames/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (int16 chirp + noise, seeded per track), resident in HBM",
            "config": {"workload": f"C5: {total} mixed-rate tracks (8-48 kHz) x {args.seconds:g} s, "
                                   f"n_fft 256-2048 per track, hop n_fft/4, amp dB + global range + "
                                   f"grey + Lanczos3 + colormap RGB at 100 px/s x 500 px",
                       "tracks_per_gpu": len(tracks), "images_per_s": total / dt,
                       "geometry_groups": len(p.groups), "frames_per_gpu": p.total_frames,
                       "ms_per_step_with_rgb_copied_to_host": dt_host * 1e3,
                       "parallelism": f"file-sharded x{ws} (LPT), one all_reduce of 3 scalars"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "spectrogram launches of all geometry groups",
                         "kernel_ms": kms, "algorithmic_bytes_per_launch": in_bytes + out_bytes},
        }), flush=True)
    p.close()


def main():
    args = parse()
    ws, rank, local, pg = dist_setup(args)
    # one rank per GPU; on a box with fewer GPUs than ranks (a rehearsal) ranks share devices
    engine.set_device(local % max(1, engine.device_count()))
    if args.workload == "c5":
        main_c5(args, ws, rank, pg)
        if pg is not None:
            pg.destroy_process_group()
        return
    n_samples = int(round(args.seconds * args.sr))
    kind = {"mel_db": engine.OUT_MEL_AMP_DB, "amp_db": engine.OUT_AMP_DB,
            "power_db": engine.OUT_POWER_DB, "complex": engine.OUT_COMPLEX}[args.output]
    fmt = engine.IN_F32 if args.input == "f32" else engine.IN_S16
    plan = engine.Plan(args.n_fft, args.n_fft, args.hop, kind, sr=args.sr,
                       n_mels=args.n_mels if kind == engine.OUT_MEL_AMP_DB else 0)
    el = 4 if fmt == engine.IN_F32 else 2
    per_track = n_samples * args.channels
    # the job's tracks (tracks-per-GPU x ranks) are partitioned per file by LPT
    # (thesia.shard); every rank computes the same partition, no exchange
    mine = shard.plan_shards([n_samples] * (args.tracks * ws), args.n_fft, args.hop, args.n_fft,
                             args.n_mels if kind == engine.OUT_MEL_AMP_DB else 0, ws, rank)
    n_local = len(mine)
    din = engine.DeviceBuffer(n_local * per_track * el)
    # distinct tracks per rank: the generator is seeded per rank and track
    engine.synth_pcm_device(din, fmt, args.channels, n_local, n_samples, args.sr, seed=rank)
    offs = np.arange(n_local, dtype=np.uint64) * per_track
    lens = np.full(n_local, n_samples, np.uint64)
    frames = engine.Batch.frames_for(plan, lens)
    dout = engine.DeviceBuffer(frames * plan.row_bins * (8 if kind == engine.OUT_COMPLEX else 4))
    batch = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=args.channels)
    assert batch.total_frames == frames

    for _ in range(args.warmup):
        batch.run()
    engine.synchronize()
    barrier(pg)
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.run()
    engine.synchronize()
    barrier(pg)
    t1 = time.perf_counter()
    dt = max_over_ranks(pg, (t1 - t0) / args.steps)

    if args.variants:
        vs = [int(v) for v in args.variants.split(",")]
        res = {v: [] for v in vs}
        for _ in range(5):  # interleaved rounds (methodology rule 24)
            for v in vs:
                os.environ["THESIA_STFT_VARIANT"] = str(v)
                batch.run_timed(1)
                res[v].append(batch.run_timed(3) / 3)
        os.environ["THESIA_STFT_VARIANT"] = "0"
        if rank == 0:
            print(json.dumps({"variants_kernel_ms": {str(v): {"median": float(np.median(t)), "min": float(min(t))}
                                                     for v, t in res.items()}}), flush=True)

    # kernel duration from HIP events on the launch stream (roofline numerator / denominator)
    kms = batch.run_timed(max(args.steps, 5)) / max(args.steps, 5)
    kms = max_over_ranks(pg, kms)
    abytes = algorithmic_bytes(args, n_local, n_samples, frames, plan.row_bins)
    achieved = abytes / (kms * 1e-3) / 1e9

    total_frames_all = frames_all_ranks(pg, frames)
    result = {
        "metric": "STFT frames/sec (n_fft=2048 hop=512) at 1/2/4/8 GPUs; % HBM roofline",
        "value": total_frames_all / dt,
        "unit": "frames/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (int16-quantised chirp + noise, seeded per track), resident in HBM",
        "config": {
            "workload": f"{args.workload.upper()} per-GPU shard: {n_local} x {args.sr/1000:g} kHz {args.seconds:g} s "
                        f"{'stereo' if args.channels == 2 else str(args.channels) + '-ch'} tracks per GPU "
                        f"({args.input} interleaved), n_fft {args.n_fft} hop {args.hop} Hann, "
                        f"sum-downmix, {'mel-' + str(args.n_mels) + ' + amp dB' if kind == engine.OUT_MEL_AMP_DB else args.output}",
            "tracks_per_gpu": n_local,
            "tracks_total": args.tracks * ws,
            "frames_per_gpu": frames,
            "parallelism": f"file-sharded x{ws}, no collective",
        },
    }
    if rank == 0:
        wkey = f"{args.output}_{args.input}_{args.channels}ch_{args.n_fft}_{args.hop}"
        result["roofline"] = {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic_from_profile(wkey),
            "kernel": {1: "thesia::stft_kernel (general)", 2: "thesia::stft2_kernel (general, 4 waves/SIMD)",
                       3: "thesia::stft3_kernel (streaming)"}.get(batch.kernel, "?")
                      + ": downmix+frame+window+rFFT+" + {"mel_db": "|X|+mel+dB", "amp_db": "|X|+dB",
                                                           "power_db": "|X|^2+dB", "complex": "complex out"}[args.output]
                      + ", one launch",
            "kernel_ms": kms,
            "algorithmic_bytes_per_launch": abytes,
        }
        if kind != engine.OUT_COMPLEX and not args.no_rfft_roofline:
            result["roofline_window_rfft"] = rfft_roofline(args, din, offs, lens, fmt, n_local, n_samples)
        if ws == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args, n_samples)
        print(json.dumps(result), flush=True)
    batch.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
