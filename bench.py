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

Launch: `python bench.py [--gpus N --steps K --warmup W]`. With --gpus N > 1 and no
WORLD_SIZE in the environment this process is only a launcher: it spawns N worker processes
(RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one per GPU) before anything touches a GPU,
relays rank 0's JSON line and exits with the workers' status. Under torch.distributed.run the
process is a worker directly. gloo carries only the timing barrier / max and the per-rank
report. Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
METRIC = "STFT frames/sec (n_fft=2048 hop=512) at 1/2/4/8 GPUs; % HBM roofline"
KERNEL_NAMES = {1: "thesia::stft_kernel (general)", 2: "thesia::stft2_kernel (general, 4 waves/SIMD)",
                3: "thesia::stft3_kernel (streaming)", 5: "thesia::stft5_kernel (streaming, n_fft 2048)",
                7: "thesia::stftr_kernel (streaming, reference order, bit-exact)",
                9: "thesia::stftx_kernel (reference order, bit-exact)"}


def kernel_name(k, n_fft):
    """Batch kernel 7 is stftr at n_fft 2048 and stftq at 256 / 512 / 1024."""
    if k == 7 and n_fft != 2048:
        return "thesia::stftq_kernel (streaming, reference order, bit-exact)"
    return KERNEL_NAMES.get(k, str(k))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--workload", choices=["c4", "c3", "c5", "viewer"], default="c4",
                   help="c4 (default, BASELINE.json metric): 48 kHz 30 s stereo, mel-128; "
                        "c3: 48 kHz 10 s mono, mel-128; c5: mixed rates / n_fft, dB + RGB render; "
                        "viewer: the reference's own four criterion benches (benches/bench.rs) "
                        "through the drop-in MultiTrack path")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--tracks", type=int, default=1000, help="tracks per GPU")
    p.add_argument("--seconds", type=float, default=None, help="default 30 (c4) / 10 (c3, c5)")
    p.add_argument("--sr", type=int, default=48000)
    p.add_argument("--channels", type=int, default=None, help="default 2 (c4) / 1 (c3, c5)")
    p.add_argument("--input", choices=["f32", "s16"], default="f32")
    p.add_argument("--n-fft", type=int, default=2048)
    p.add_argument("--hop", type=int, default=512)
    p.add_argument("--win", type=int, default=None,
                   help="window length (default n_fft; the viewer geometries: e.g. 1920 with --hop 480)")
    p.add_argument("--n-mels", type=int, default=128)
    p.add_argument("--output", choices=["mel_db", "amp_db", "power_db", "complex"], default="mel_db")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-exact", action="store_true",
                   help="c4: skip the bit-exact (reference-order kernel 7) line reported beside the default "
                        "one; c5: time the tolerance kernels as the line's path (default: kernel 7, the "
                        "tolerance path beside it)")
    p.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive end-to-end sample")
    p.add_argument("--no-rfft-roofline", action="store_true",
                   help="skip the extra complex-output (window+rFFT kernel) roofline measurement")
    p.add_argument("--no-c1", action="store_true", help="skip the C1 (48 kHz sample, 1024/256) line")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU baseline threads (0: OMP_NUM_THREADS if set, else the affinity mask)")
    p.add_argument("--variants", default="", help="experiment (needs THESIA_LIB=lib/libthesia_exp.so): "
                   "comma list of THESIA_STFT_VARIANT values to A/B (interleaved rounds, one process)")
    p.add_argument("--kernel", type=int, default=0, help="force a fused kernel (1/2/3/5; 7 / 9 = the bit-exact "
                   "reference-order kernels, streaming / one wave per frame; 0 = automatic)")
    p.add_argument("--max-blocks", default="", help="A/B of the launch's block count (thesia_batch_set_option "
                   "MAX_BLOCKS): comma list, 0 = the occupancy default")
    p.add_argument("--kernels", default="", help="A/B of named kernels on the product library: comma list "
                   "of kernel ids (interleaved rounds, one process), e.g. 3,5")
    p.add_argument("--mel-paths", default="", help="A/B of stft5's mel projections (THESIA_BATCH_OPT_MEL_PATH): "
                   "comma list, e.g. 1,2,3 (interleaved rounds, one process)")
    p.add_argument("--row-store", type=int, default=0,
                   help="complex-output row store of the window+rFFT roofline (THESIA_BATCH_OPT_ROW_STORE, "
                        "thesia.h: 0 default = whole 128-byte lines, 1 LDS-staged 16-byte, 2 whole 128-byte "
                        "lines, 3 lane-wise 8-byte)")
    p.add_argument("--row-stores", default="", help="A/B of the complex-output row stores (comma list, "
                   "interleaved rounds, one process), reported in roofline_window_rfft")
    p.add_argument("--spec-policies", default="", help="c5: A/B of thesia_set_batches_policy for the "
                   "spectrogram phase (comma list, interleaved rounds, one process)")
    p.add_argument("--render-path", type=int, default=-1, help="c5: the display launch structure "
                   "(thesia_set_render_path; -1 = the library default)")
    p.add_argument("--render-paths", default="", help="c5: A/B of the display launch structures "
                   "(thesia_set_render_path), comma list, interleaved rounds")
    p.add_argument("--selftest", action="store_true",
                   help="launcher / reduction plumbing only: no GPU, no thesia (CPU tests)")
    p.add_argument("--selftest-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    a = p.parse_args()
    if a.win is None:
        a.win = a.n_fft
    if a.seconds is None:
        a.seconds = 30.0 if a.workload == "c4" else 10.0
    if a.channels is None:
        a.channels = 2 if a.workload == "c4" else 1
    return a


# ------------------------------------------------------------------------------------------
# launcher (no GPU, no thesia / torch import: the workers own the devices)
# ------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int) -> int:
    """Spawn n worker processes of this script (one per GPU, RANK = LOCAL_RANK = i), relay
    rank 0's stdout, wait for all; a failing worker stops the others (their exact PIDs)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    import threading

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode())
            sys.stdout.flush()

    reader = threading.Thread(target=relay, daemon=True)
    reader.start()
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:  # stop the rest: their own PIDs only
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
        reader.join(timeout=10)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc if rc >= 0 else 128 - rc


# ------------------------------------------------------------------------------------------
# worker side
# ------------------------------------------------------------------------------------------
def dist_setup():
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


def gather_reports(pg, rep: dict) -> list:
    """Every rank's report (device, frames, ...) on every rank (gloo)."""
    if pg is None:
        return [rep]
    out = [None] * pg.get_world_size()
    pg.all_gather_object(out, rep)
    return out


def ranks_summary(reports: list, frames_key: str = "frames") -> dict:
    devices = sorted({r["device"] for r in reports})
    return {"n_devices": len(devices), "devices": devices,
            "per_rank_frames": [int(r[frames_key]) for r in reports],
            "total_frames": int(sum(r[frames_key] for r in reports))}


def cpu_info() -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_threads(args) -> int:
    """The host share this run may use: --cpu-threads, else OMP_NUM_THREADS (the GPU box sets
    it to its 16-CPU share per GPU; nproc there counts the whole machine), else the affinity."""
    if args.cpu_threads > 0:
        return args.cpu_threads
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)


def cpu_baseline(args, n_samples):
    """The oracle (oracle/thesia_oracle.c, a C restatement of the reference path, test
    infrastructure) timed on a bounded sample of the same workload with the reference's
    execution structure: per-track parallel over a thread pool (rayon par_iter, lib.rs:161-166),
    one FFT plan per track (lib.rs:459-467), dense mel dot, three-pass dB. One C call per
    track (ctypes releases the GIL)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_ffi as O
    from concurrent.futures import ThreadPoolExecutor
    from thesia import engine

    threads = cpu_threads(args)
    n_tracks = 4 * threads  # ~0.19 s of CPU per C4 track: ~12 s of CPU work on 16 threads
    kind = {"mel_db": O.TRACK_MEL_DB, "amp_db": O.TRACK_AMP_DB, "power_db": O.TRACK_POWER_DB,
            "complex": O.TRACK_MAG}[args.output]
    fb = O.calc_mel_fb(args.sr, args.n_fft, args.n_mels) if kind == O.TRACK_MEL_DB else None
    pcm = [(engine.synth_pcm_host(args.channels, i, n_samples, args.sr).astype(np.float32) / np.float32(32768.0))
           for i in range(n_tracks)]

    def one(x):
        return O.track_spec(x, args.win, args.hop, args.n_fft, kind, fb).shape[0]

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        frames = sum(ex.map(one, pcm))
    dt = time.perf_counter() - t0
    return dict({"value": frames / dt, "unit": "frames/s", "cores": threads, "kind": "port",
                 "sample": f"{n_tracks} tracks x {args.seconds:g} s x {args.channels} ch @ {args.sr} Hz "
                           f"({frames} frames, {dt:.2f} s wall, {threads} threads) through the C oracle "
                           f"(one FFT plan per track, dense mel dot)"}, **cpu_info())


def c1_line(args):
    """BASELINE.json configs[0] (C1): the 48 kHz sample (substitute: tests/fixtures.py
    c1_substitute, 2 113 529 samples), n_fft 1024 / hop 256 / Hann, |X| (lib.rs:124).
    GPU: one batch of that one track (stft3_kernel), HIP-event time. CPU: the reference's
    single-track path -- frames built serially, then per-frame parallel with a fresh RealFFT
    per frame (lib.rs:449-458) over the thread pool -- through the oracle."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import fixtures
    import oracle_ffi as O
    from concurrent.futures import ThreadPoolExecutor
    from thesia import engine

    x = fixtures.s16_to_f32(fixtures.c1_substitute())
    n = x.shape[0]
    plan = engine.Plan(1024, 1024, 256, engine.OUT_MAG, sr=48000)
    din = engine.DeviceBuffer.from_host(x)
    T = engine.Batch.frames_for(plan, [n])
    dout = engine.DeviceBuffer(T * plan.row_bins * 4)
    b = engine.Batch(plan, din, [0], [n], dout)
    b.run_timed(3)
    kms = b.run_timed(20) / 20
    gpu = {"frames": T, "kernel_ms": kms, "frames_per_s": T / (kms * 1e-3), "kernel": b.kernel}
    b.close()
    dout.close()
    din.close()
    plan.close()
    out = {"workload": "C1: 48 kHz sample substitute (2 113 529 samples), n_fft 1024 hop 256 Hann, |X|",
           "gpu": gpu}
    if not args.no_cpu_baseline:
        threads = cpu_threads(args)
        reps = 8
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            for _ in range(reps):
                fr = O.frames(x, 1024, 256, 1024)
                mag = np.empty((fr.shape[0], 513), np.float32)
                step = (fr.shape[0] + threads - 1) // threads
                list(ex.map(lambda t: O.rfft_mag_rows(fr, t, min(t + step, fr.shape[0]), mag, True),
                            range(0, fr.shape[0], step)))
        dt = time.perf_counter() - t0
        out["cpu_baseline_c1"] = dict({"value": reps * T / dt, "unit": "frames/s", "cores": threads,
                                       "kind": "port",
                                       "sample": f"{reps} passes over the whole C1 track ({reps * T} frames, "
                                                 f"{dt:.2f} s wall): serial framing + per-frame parallel rfft "
                                                 f"with a RealFFT::new per frame (lib.rs:449-458) + hypot"},
                                      **cpu_info())
    return out


def algorithmic_bytes(args, n_tracks, n_samples, total_frames, row_bins):
    """Bytes one launch must move at least: the input once (hop-strided, not n_fft per frame)
    plus the output rows (DESIGN.md §4 'Roofline and algorithmic bytes')."""
    in_el = 4 if args.input == "f32" else 2
    out_el = 8 if args.output == "complex" else 4
    return n_tracks * n_samples * args.channels * in_el + total_frames * row_bins * out_el


def hbm_ceiling(din, in_bytes, dout, out_bytes):
    """The box's own ceiling for a kernel's read : write mix, measured in this process on the
    kernel's own two buffers (thesia_hbm_ceiling: the input read once and the output written
    once by a coalesced float4 copy, best of 3 x 2 grid sizes)."""
    import ctypes as C
    from thesia._lib import lib, check
    ms, gbps = C.c_float(), C.c_float()
    check(lib.thesia_hbm_ceiling(din.ptr, C.c_size_t(in_bytes), dout.ptr, C.c_size_t(out_bytes), 3,
                                 C.byref(ms), C.byref(gbps)))
    return {"ceiling_gbs": gbps.value, "ceiling_ms": ms.value,
            "ceiling": "thesia_hbm_ceiling on the same buffers in this process: the input read once and "
                       "the output written once by a coalesced float4 copy (best of 3 x 2 grid sizes)"}


_TORCH_CEILING = r"""
import json, sys, torch
n_in, n_out, dev = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
torch.cuda.set_device(dev)
x = torch.ones(n_in, device="cuda", dtype=torch.float32)
y = torch.empty(n_out, device="cuda", dtype=torch.float32)
n = n_out // 2
src, dst = x[:n].view(n, 1).expand(n, 2), y[:2 * n].view(n, 2)
dst.copy_(src)
torch.cuda.synchronize()
best = None
for _ in range(3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        dst.copy_(src)
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / 3
    best = ms if best is None else min(best, ms)
print(json.dumps({"ms": best, "bytes": 12 * n}))
"""


def torch_ceiling(in_bytes, out_bytes, device):
    """PyTorch's own copy kernel for the kernel's read : write mix (scripts/hbm_rates.py
    'read1_write2'): every input float read once and written twice, y[i, 0:2] = x[i], buffers of
    the kernel's sizes; HIP events on torch's stream, best of 3 rounds of 3 (VERDICT r04 item 4:
    the box's best copy next to thesia_hbm_ceiling). A child process: torch bundles its own HIP
    runtime, which sees no device inside a process where libthesia's runtime is already up."""
    n_in = in_bytes // 4
    n_out = min(out_bytes // 4, 2 * n_in)
    r = subprocess.run([sys.executable, "-c", _TORCH_CEILING, str(n_in), str(n_out), str(device)],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError((r.stderr or r.stdout).strip()[-300:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {"torch_ceiling_gbs": d["bytes"] / (d["ms"] * 1e-3) / 1e9, "torch_ceiling_ms": d["ms"],
            "torch_ceiling_bytes": d["bytes"],
            "torch_ceiling": "PyTorch copy_ of an input of the kernel's input size into an output of its "
                             "size as [n, 2] (each float read once, written twice), a child process on the "
                             "same device while this one holds its buffers, best of 3 x 3"}


def ab_row_stores(args, b):
    import numpy as np
    from thesia import engine
    rs = [int(v) for v in args.row_stores.split(",")]
    t = {q: [] for q in rs}
    for _ in range(5):  # interleaved rounds
        for q in rs:
            b.set_option(engine.OPT_ROW_STORE, q)
            b.run_timed(1)
            t[q].append(b.run_timed(3) / 3)
    b.set_option(engine.OPT_ROW_STORE, args.row_store)
    return {str(q): {"median": float(np.median(v)), "min": float(min(v))} for q, v in t.items()}


def rfft_roofline(args, din, offs, lens, fmt, n_local, n_samples):
    """BASELINE.json north_star's "window+rFFT kernel" on the same resident input: the same
    streaming kernel with complex-spectrum output ([T, F] complex64, perform_stft's result,
    lib.rs:436-440), timed with HIP events on its launch stream; algorithmic bytes = input once
    + F x 8 B per frame. Beside it the box's own ceiling for that read : write mix, measured in
    this process on the same two buffers (thesia_hbm_ceiling: every input byte read once, every
    output byte written once, coalesced float4). Reported beside the headline roofline, never as
    `value`."""
    from thesia import engine
    plan = engine.Plan(args.n_fft, args.win, args.hop, engine.OUT_COMPLEX, sr=args.sr)
    frames = engine.Batch.frames_for(plan, lens)
    out_bytes = frames * plan.row_bins * 8
    dout = engine.DeviceBuffer(out_bytes)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=args.channels,
                     kernel=args.kernel, row_store=args.row_store)
    b.run_timed(2)
    kms = b.run_timed(5) / 5
    kname = kernel_name(b.kernel, args.n_fft)
    in_el = 4 if args.input == "f32" else 2
    in_bytes = n_local * n_samples * args.channels * in_el
    abytes = in_bytes + out_bytes
    achieved = abytes / (kms * 1e-3) / 1e9
    res = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "kernel_ms": kms, "algorithmic_bytes_per_launch": abytes,
           "frames_per_s": frames / (kms * 1e-3), "row_store": args.row_store,
           "kernel": kname + ", complex output (downmix+frame+window+rFFT)"}
    if args.row_stores:
        res["row_stores_ms"] = ab_row_stores(args, b)
    res.update(hbm_ceiling(din, in_bytes, dout, out_bytes))
    try:
        from thesia import engine
        res.update(torch_ceiling(in_bytes, out_bytes, engine.current_device()))
    except Exception as e:  # noqa: BLE001 (reported, the line stands without it)
        res["torch_ceiling_error"] = repr(e)[:200]
    best = max(res["ceiling_gbs"], res.get("torch_ceiling_gbs", 0.0))
    res["frac_of_ceiling"] = achieved / best
    res["frac_of_ceiling_note"] = "against the faster of thesia_hbm_ceiling and the PyTorch copy"
    res["frac_of_thesia_ceiling"] = achieved / res["ceiling_gbs"]
    b.close()
    dout.close()
    return res


def workload_params(args, kernel):
    """Every parameter that changes what one launch moves or issues (the key of a stored PMC
    record: a record applies to this run only if all of them are equal)."""
    return {"output": args.output, "input": args.input, "channels": args.channels, "n_fft": args.n_fft,
            **({"win": args.win} if args.win != args.n_fft else {}),
            "hop": args.hop, "tracks_per_gpu": args.tracks, "seconds": args.seconds, "sr": args.sr,
            "n_mels": args.n_mels if args.output == "mel_db" else 0, "kernel": kernel, "mel_path": 0}


def profile_record(params):
    """The PMC record of profiles/pmc_traffic.json measured on exactly this workload, or None.
    Its counts come from a rocprofv3 run on a builder box (the file names the profile), not from
    this run: the bench line says so next to every value it takes from it."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            recs = json.load(f)
    except (OSError, ValueError):
        return None
    for rec in recs.values():
        if rec.get("workload") == params:
            return rec
    return None


def provenance(rec):
    out = {"profile": "profiles/" + rec.get("profile", "?"), "date": rec.get("date"), "box": rec.get("box"),
           "measured_in_this_run": False,
           "note": "stored rocprofv3 PMC counts of the same workload from a builder box "
                   "(profiles/pmc_traffic.json), not measured by this run"}
    latest = rec.get("reconfirmed_round6")
    if latest:  # the latest re-measurement of the same counters on the current kernels
        out["reconfirmed"] = {"profile": "profiles/" + latest.get("profile", "?"), "note": latest.get("note")}
    return out


# VALU issue ceiling (MI355X_MICROARCH.md constants table): a wave64 v_fma_f32 occupies its
# SIMD-32 for 2 cycles, 4 SIMDs per CU, 256 CUs, 2.4 GHz peak engine clock
VALU_ISSUE_PEAK_G = 256 * 4 * 2.4e9 / 2 / 1e9  # wave-instructions per second, in G


def issue_ceiling(rec, kms):
    """The mel kernel's other roofline: its VALU wave-instructions per launch (a PMC count of
    the kernel on this exact workload, profiles/pmc_traffic.json) over the live kernel time,
    against the chip's VALU issue peak. DESIGN.md §7: the kernel is issue-bound, not HBM-bound."""
    n = rec.get("valu_insts_per_launch") if rec else None
    if n is None:
        return None
    achieved = n / (kms * 1e-3) / 1e9
    return {"bound": "valu-issue", "achieved": achieved, "peak": VALU_ISSUE_PEAK_G,
            "unit": "G wave-instructions/s", "frac": achieved / VALU_ISSUE_PEAK_G,
            "valu_insts_per_launch": n, "valu_insts_source": provenance(rec)}


def main_selftest(args, ws, rank, pg):
    """Launcher plumbing without a GPU: each rank 'processes' (rank + 1) x 1000 frames in a
    short sleep; the reductions are the real ones (gloo barrier, max time, report gather)."""
    if rank == args.selftest_fail_rank:
        sys.exit(3)
    barrier(pg)
    t0 = time.perf_counter()
    time.sleep(0.05 * (rank + 1))
    barrier(pg)
    dt = max_over_ranks(pg, time.perf_counter() - t0)
    reps = gather_reports(pg, {"device": rank, "frames": 1000 * (rank + 1), "pid": os.getpid()})
    if rank == 0:
        s = ranks_summary(reps)
        print(json.dumps({"selftest": True, "n_ranks": ws, "n_gpus": s["n_devices"], "value": s["total_frames"] / dt,
                          "ms_per_step": dt * 1e3, "per_rank_frames": s["per_rank_frames"],
                          "pids": [r["pid"] for r in reps]}), flush=True)


def main_c5(args, ws, rank, pg, device):
    """C5 (BASELINE.json configs[4]): mixed-rate tracks with per-track n_fft, amp dB, global
    range exchange, grey + Lanczos3 + colormap RGB for every track (thesia.pipeline). One step =
    spectrogram launches for every geometry group + the display path of every track, the RGB
    images left in HBM (the copy to the host that get_spec_image implies, lib.rs:294-298, is
    timed separately: PCIe-inclusive, never the reported value)."""
    from thesia import engine, pipeline, shard

    total = args.tracks * ws
    gen = pipeline.c5_tracks(total, seconds=0.0)  # geometry only (empty PCM) for the partition
    # both phases balanced (the display waits for every rank's range: a step pays the slowest
    # rank of each phase), thesia.shard.assign_tracks_2phase
    lens = [int(round(args.seconds * t.sr)) for t in gen]
    max_sr = max(t.sr for t in gen)
    spec_costs = [shard.track_cost(n, t.n_fft, t.n_fft // 4, t.n_fft) for n, t in zip(lens, gen)]
    disp_costs = [shard.display_cost(n, t.sr, t.n_fft, t.n_fft // 4, t.n_fft, max_sr, 100.0, 500)
                  for n, t in zip(lens, gen)]
    mine = shard.assign_tracks_2phase(spec_costs, disp_costs, ws)[rank]
    tracks = []
    for i in mine:  # the generator is indexed by the global track id
        tracks += pipeline.c5_tracks(1, seconds=args.seconds, first=i, channels=args.channels)
    if args.render_path >= 0:
        engine.set_render_path(args.render_path)
    p = pipeline.RenderPipeline(tracks, px_per_sec=100.0, nheight=500, pinned_output=True, kernel=args.kernel)

    def step(want_rgb=False):
        # images stay in HBM in the timed step (inputs resident, outputs resident); the
        # host-copy-inclusive rate is measured separately below
        p.run_spectrograms()
        p.render(group=None, want_rgb=want_rgb)

    def use_kernel(k):
        for _, _, _, b in p.groups:
            b.set_option(engine.OPT_KERNEL, k)

    def timed_steps(k, warm, n):
        use_kernel(k)
        for _ in range(warm):
            step()
        engine.synchronize()
        barrier(pg)
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        engine.synchronize()
        barrier(pg)
        return max_over_ranks(pg, (time.perf_counter() - t0) / n)

    def spectrogram_phase():
        # each batch's launch alone (HIP events per launch), and the step's spectrogram phase as
        # it runs: the batches overlapped on the library streams
        alone = [(pl.n_fft, b.total_frames, b.run_timed(3) / 3, b.kernel) for pl, _, _, b in p.groups]
        engine.synchronize()
        p.run_spectrograms()
        with engine.EventTimer() as tm:
            for _ in range(3):
                p.run_spectrograms()
        return alone, tm.ms / 3

    # The line's path: north_star asks for the final u8 RGB bytes equal to the reference's, so the
    # reported step runs every batch on the reference-order streaming kernels (7: stftq at n_fft
    # 256 / 512 / 1024, stftr at 2048; RGB bytes equal to the oracle pipeline's,
    # tests/test_gpu_parity.py test_e2e_rgb_c5_generator_exact); the tolerance kernels' step is
    # reported beside it (tolerance_path). --kernel K / --no-exact measure that path instead.
    main_k = 7 if (args.kernel == 0 and not args.no_exact) else args.kernel
    dt = timed_steps(main_k, args.warmup, args.steps)
    step(want_rgb=True)  # untimed: pins the host readback buffers once (hipHostRegister)
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        step(want_rgb=True)
    engine.synchronize()
    dt_host = max_over_ranks(pg, (time.perf_counter() - t0) / 3)
    kms_batches, kms_overlap = spectrogram_phase()
    kms = sum(t for _, _, t, _ in kms_batches)
    tol = None
    if main_k == 7:
        tol_dt = timed_steps(0, 2, args.steps)
        tol_batches, tol_overlap = spectrogram_phase()
        tol = {"kernel": 0, "ms_per_step": tol_dt * 1e3, "frames_per_s": p.total_frames / tol_dt,
               "spectrogram_overlapped_ms": tol_overlap,
               "spectrogram_kernel_ms": sum(t for _, _, t, _ in tol_batches),
               "per_batch": [{"n_fft": nf, "kernel_ms": t, "kernel": kernel_name(k, nf)} for nf, _, t, k in tol_batches],
               "exact_over_tolerance_step": dt / tol_dt,
               "note": "the automatic (tolerance) kernels: rows within the stated fp32 tolerance of the "
                       "oracle, RGB within the fast path's end-to-end contract (not bit-exact)"}
        use_kernel(main_k)
    disp = p.display_timed(3)
    # the display's stored PMC record (this geometry, one GPU, render path 0): HBM traffic beside
    # the algorithmic bytes, and its VALU issue roofline (the passes are issue- and
    # latency-bound; the f32 intermediate of the two-kernel groups and the halo re-reads are the
    # traffic above algorithmic)
    drec = profile_record({"workload": "c5_display", "tracks": total, "seconds": args.seconds,
                           "px_per_sec": 100.0, "nheight": 500, "render_path": max(args.render_path, 0)}) \
        if ws == 1 else None
    disp.pop("traffic_note", None)
    disp["traffic"] = drec["hbm_bytes_per_launch"] if drec else None
    disp["traffic_source"] = provenance(drec) if drec else "no stored PMC record of this exact workload"
    disp_ic = issue_ceiling(drec, disp["display_ms"]) if drec else None
    spec_ceiling = None
    if ws == 1:
        # each phase's same-process copy ceiling: the display's algorithmic
        # bytes (the dB rows read once, the RGB written once) and the spectrogram phase's (PCM read
        # once, rows written once) moved by thesia_hbm_ceiling's coalesced float4 copy
        db = disp["algorithmic_bytes"]
        scratch = engine.DeviceBuffer(db["spec_read"])
        disp.update(hbm_ceiling(scratch, db["spec_read"], p._rgb, db["rgb_write"]))
        disp["frac_of_ceiling"] = disp["achieved"] / disp["ceiling_gbs"]
        scratch.close()
        sin = sum(t.pcm.nbytes for t in tracks)
        sout = sum(b.total_frames * pl.row_bins * 4 for pl, _, _, b in p.groups)
        s_in, s_out = engine.DeviceBuffer(sin), engine.DeviceBuffer(sout)
        spec_ceiling = hbm_ceiling(s_in, sin, s_out, sout)
        s_in.close()
        s_out.close()
    pol_ms = None
    if args.spec_policies:
        import numpy as np
        pols = [int(v) for v in args.spec_policies.split(",")]
        res = {q: [] for q in pols}
        for _ in range(5):  # interleaved rounds
            for q in pols:
                engine.set_batches_policy(q)
                p.run_spectrograms()
                with engine.EventTimer() as tm:
                    for _ in range(3):
                        p.run_spectrograms()
                res[q].append(tm.ms / 3)
        engine.set_batches_policy(0)
        pol_ms = {str(q): {"median": float(np.median(t)), "min": float(min(t))} for q, t in res.items()}
    mb_ms = None
    if args.max_blocks:  # per batch, each alone: its launch's block count (0 = occupancy default)
        import numpy as np
        ms = [int(v) for v in args.max_blocks.split(",")]
        res = {(pl.n_fft, m): [] for pl, _, _, _ in p.groups for m in ms}
        for _ in range(5):  # interleaved rounds
            for pl, _, _, b in p.groups:
                for m in ms:
                    b.set_option(engine.OPT_MAX_BLOCKS, m)
                    res[(pl.n_fft, m)].append(b.run_timed(3) / 3)
        for _, _, _, b in p.groups:
            b.set_option(engine.OPT_MAX_BLOCKS, 0)
        mb_ms = {str(nf): {str(m): float(np.median(res[(nf, m)])) for m in ms} for nf in sorted({k[0] for k in res})}
    if args.render_paths:
        import numpy as np
        rp = [int(v) for v in args.render_paths.split(",")]
        res = {q: [] for q in rp}
        for _ in range(5):  # interleaved rounds
            for q in rp:
                engine.set_render_path(q)
                res[q].append(p.display_timed(3)["display_ms"])
        engine.set_render_path(max(args.render_path, 0))
        if rank == 0:
            print(json.dumps({"render_paths_ms": {str(q): {"median": float(np.median(t)), "min": float(min(t))}
                                                  for q, t in res.items()}}), flush=True)
    in_bytes = sum(t.pcm.nbytes for t in tracks)
    out_bytes = sum(b.total_frames * pl.row_bins * 4 for pl, _, _, b in p.groups)
    achieved = (in_bytes + out_bytes) / (kms * 1e-3) / 1e9
    reps = gather_reports(pg, {"device": device, "frames": p.total_frames, "tracks": len(tracks)})
    summ = ranks_summary(reps)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": summ["total_frames"] / dt, "unit": "frames/s", "n_gpus": summ["n_devices"], "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (int16 chirp + noise, seeded per track), resident in HBM",
            "config": {"workload": f"C5: {total} mixed-rate tracks (8-48 kHz) x {args.seconds:g} s, "
                                   f"n_fft 256-2048 per track, hop n_fft/4, amp dB + global range + "
                                   f"grey + Lanczos3 + colormap RGB at 100 px/s x 500 px",
                       "ranks": ws, "devices": summ["devices"], "per_rank_frames": summ["per_rank_frames"],
                       "tracks_per_gpu": len(tracks), "images_per_s": total / dt,
                       "spectrogram_batches": len(p.groups), "display_groups": p._n_disp,
                       "frames_per_gpu": p.total_frames,
                       "spectrogram_path": (f"kernel {main_k}: reference-order streaming kernels (stftq at n_fft "
                                            f"256-1024, stftr at 2048), RGB bytes equal to the oracle pipeline's"
                                            if main_k == 7 else f"kernel {main_k} (0 = automatic, tolerance)"),
                       "ms_per_step_with_rgb_copied_to_host": dt_host * 1e3,
                       "parallelism": f"file-sharded x{ws} (LPT), one all_reduce of 3 scalars"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "spectrogram launches of all geometry groups",
                         "kernel_ms": kms, "algorithmic_bytes_per_launch": in_bytes + out_bytes,
                         "kernel_ms_note": "sum of the batches' launches, each timed alone",
                         "overlapped_ms": kms_overlap,
                         "copy_ceiling": spec_ceiling,
                         "frac_of_ceiling": ((in_bytes + out_bytes) / (kms_overlap * 1e-3) / 1e9 / spec_ceiling["ceiling_gbs"])
                                            if spec_ceiling else None,
                         "batches_policy_ms": pol_ms,
                         "per_batch_max_blocks_ms": mb_ms,
                         "per_batch": [{"n_fft": nf, "frames": fr, "kernel_ms": t, "kernel": kernel_name(k, nf)}
                                       for nf, fr, t, k in kms_batches],
                         "overlapped_note": "the step's spectrogram phase: the batches on the library "
                                            "streams (thesia_batches_run), HIP events on the library stream"},
            "tolerance_path": tol,
            "roofline_display": disp,
            "roofline_display_valu_issue": disp_ic,
        }), flush=True)
    p.close()


def _median_s(fn, reps, warm=1):
    import numpy as np
    from thesia import engine
    for _ in range(warm):
        fn()
    engine.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        engine.synchronize()
        t.append(time.perf_counter() - t0)
    return float(np.median(t))


def main_viewer(args, rank):
    """The reference's own measurement spec, benches/bench.rs (criterion; it does not compile at
    this revision, bench.rs:86, and reads the absent samples/sample.wav: the 48 kHz substitute
    of tests/fixtures.py stands in). Four entries, each with the GPU time of the drop-in path
    and the oracle's CPU time beside it:
      get_melspectrogram  bench.rs:7-25,62-77: 1 s @ 48 kHz, win 1920 / hop 480 / n_fft 2048
                          (the viewer geometry, lib.rs:43-46), default n_mel, amp dB
      draw_spec           bench.rs:79-95: grey -> Lanczos3 + colormap RGB, 100 px/s x 500
      add_tracks          bench.rs:32-45: MultiTrack.add_tracks of the sample six times (ids 0-5)
      get_spec_image      bench.rs:47-60: get_spec_image(0, 100, 500) after that add
    plus the kernels behind add_tracks on the same six tracks: the reference-order stftx
    (MultiTrack's, bit-exact) and the batch engine's fast kernel for that geometry."""
    import tempfile
    import wave
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import fixtures
    import oracle_ffi as O
    import thesia
    from thesia import engine, display

    sr, win, hop, n_fft = 48000, 1920, 480, 2048
    pcm16 = fixtures.c1_substitute()
    x_full = fixtures.s16_to_f32(pcm16)
    x1 = x_full[:sr]  # bench.rs:66 slice ..sr
    fb = O.calc_mel_fb_default(sr, n_fft)
    n_mel = fb.shape[1]
    out = {"metric": "viewer drop-in path: the four criterion benches of benches/bench.rs, GPU vs oracle CPU",
           "unit": "ms per call", "higher_is_better": False, "dtype": "f32",
           "data": "tests/fixtures.py c1_substitute (the 48 kHz sample stand-in, 2 113 529 samples, int16 WAV)",
           "config": {"workload": "viewer", "sr": sr, "win": win, "hop": hop, "n_fft": n_fft, "n_mel_default": n_mel},
           "entries": {}}
    E = out["entries"]

    # -- get_melspectrogram: 1 s, reference-order kernel and the fast kernel, kernel-only and host-in/out
    plan = engine.Plan(n_fft, win, hop, engine.OUT_MEL_AMP_DB, sr=sr)
    din = engine.DeviceBuffer.from_host(x1)
    T1 = engine.Batch.frames_for(plan, [len(x1)])
    dout = engine.DeviceBuffer(T1 * plan.row_bins * 4)
    ent = {"frames": T1, "n_mel": plan.row_bins}
    for name, k in (("kernel 7 (reference order, bit-exact; MultiTrack default)", 7),
                    ("stftx (reference order, bit-exact)", 9), ("fast kernel", 0)):
        b = engine.Batch(plan, din, [0], [len(x1)], dout, kernel=k)
        b.run_timed(3)
        kms = b.run_timed(50) / 50
        host = np.empty((T1, plan.row_bins), np.float32)

        def call():  # host PCM in, host dB rows out (what perform_stft + dot + dB hand back)
            from thesia._lib import lib, check
            import ctypes as C
            check(lib.thesia_memcpy_h2d(din.ptr, x1.ctypes.data_as(C.c_void_p), x1.nbytes))
            b.run()
            check(lib.thesia_memcpy_d2h(host.ctypes.data_as(C.c_void_p), dout.ptr, host.nbytes))
        ent[name] = {"kernel": b.kernel, "kernel_ms": kms, "call_ms_host_in_out": 1e3 * _median_s(call, 50)}
        b.close()
    t_cpu = _median_s(lambda: O.track_spec(x1, win, hop, n_fft, O.TRACK_MEL_DB, fb), 20)
    ent["cpu_oracle_ms"] = 1e3 * t_cpu
    ent["cpu"] = "oracle track_spec, 1 thread (one FFT plan, dense mel dot, 3-pass dB)"
    E["get_melspectrogram"] = ent
    spec = O.track_spec(x1, win, hop, n_fft, O.TRACK_MEL_DB, fb)

    # -- draw_spec: grey of that spectrogram (up_ratio 1) -> RGB 100 px/s x 500
    grey = O.spec_to_grey(spec, 1.0, float(spec.max()), float(spec.min()))
    nw = 100 * len(x1) // sr
    dgrey = engine.DeviceBuffer.from_host(grey)
    drgb = engine.DeviceBuffer(nw * 500 * 3)
    from thesia._lib import lib, check
    g_dev = _median_s(lambda: check(lib.thesia_grey_to_rgb_device(dgrey.ptr, grey.shape[1], grey.shape[0],
                                                                  nw, 500, drgb.ptr)), 50)
    g_host = _median_s(lambda: display.grey_to_rgb(grey, nw, 500), 20)
    E["draw_spec"] = {"nwidth": nw, "nheight": 500, "gpu_ms_device_buffers": 1e3 * g_dev,
                      "gpu_ms_host_in_out": 1e3 * g_host,
                      "cpu_oracle_ms": 1e3 * _median_s(lambda: O.grey_to_rgb(grey, nw, 500), 10)}

    # -- add_tracks x6 and get_spec_image through MultiTrack, from a WAV file like the reference
    tmp = tempfile.mkdtemp(prefix="thesia_viewer_")
    path = os.path.join(tmp, "sample.wav")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes(pcm16.astype("<i2").tobytes())
    mt = thesia.MultiTrack()
    ids = [0, 1, 2, 3, 4, 5]
    paths = "\n".join([path] * 6)
    t_add = _median_s(lambda: mt.add_tracks(ids, paths), 5)
    nwi = int(np.float32(100.0) * np.float32(len(x_full)) / np.float32(sr))
    t_img = _median_s(lambda: mt.get_spec_image(0, 100.0, 500), 10)
    # the CPU side: the reference's structure, one track per rayon worker (lib.rs:161-166)
    from concurrent.futures import ThreadPoolExecutor

    def cpu_add():
        with ThreadPoolExecutor(6) as ex:
            specs = list(ex.map(lambda _: O.track_spec(x_full, win, hop, n_fft, O.TRACK_MEL_DB, fb), ids))
        mx = min(max(float(v.max()) for v in specs), 0.0)
        mn = max(min(float(v.min()) for v in specs), mx - 120.0)
        with ThreadPoolExecutor(6) as ex:
            return list(ex.map(lambda v: O.spec_to_grey(v, 1.0, mx, mn), specs))
    t0 = time.perf_counter()
    greys = cpu_add()
    t_cpu_add = time.perf_counter() - t0
    t_cpu_img = _median_s(lambda: O.grey_to_rgb(greys[0], nwi, 500), 3)
    E["add_tracks"] = {"tracks": 6, "samples_per_track": len(x_full), "gpu_ms": 1e3 * t_add,
                       "gpu": "MultiTrack.add_tracks: WAV parse + int16 upload + decode + kernel 7 (bit-exact) + range + "
                              "grey, synchronous",
                       "cpu_oracle_ms": 1e3 * t_cpu_add, "cpu_threads": 6,
                       "cpu": "oracle track_spec per track on 6 threads (rayon par_iter, lib.rs:161-166) + range + "
                              "spec_to_grey; no WAV parse"}
    E["get_spec_image"] = {"nwidth": nwi, "nheight": 500, "gpu_ms": 1e3 * t_img,
                           "gpu": "MultiTrack.get_spec_image: Lanczos3 + colormap on the device + RGB copy to the host",
                           "cpu_oracle_ms": 1e3 * t_cpu_img, "cpu": "oracle grey_to_rgb, 1 thread"}
    del mt
    os.remove(path)
    os.rmdir(tmp)

    # -- the kernels behind add_tracks on the same six tracks: the mono f32 pool MultiTrack's
    # decode fills (its batch input), one launch over the six
    n = len(pcm16)
    flat = np.concatenate([x_full] * 6)
    din6 = engine.DeviceBuffer.from_host(flat)
    offs = [i * n for i in range(6)]
    T6 = engine.Batch.frames_for(plan, [n] * 6)
    dout6 = engine.DeviceBuffer(T6 * plan.row_bins * 4)
    kk = {}
    for name, k in (("kernel7", 7), ("stftx", 9), ("fast", 0)):
        b = engine.Batch(plan, din6, offs, [n] * 6, dout6, kernel=k)
        b.run_timed(2)
        kms = b.run_timed(10) / 10
        abytes = flat.nbytes + T6 * plan.row_bins * 4
        kk[name] = {"kernel": b.kernel, "kernel_ms": kms, "frames_per_s": T6 / (kms * 1e-3),
                    "algorithmic_gbs": abytes / (kms * 1e-3) / 1e9,
                    "hbm_frac": abytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        b.close()
    E["add_tracks_kernels"] = dict(kk, frames=T6, algorithmic_bytes=flat.nbytes + T6 * plan.row_bins * 4,
                                   note="kernel7 is MultiTrack's default (bit-exact, round 6: streaming "
                                        "reference-order kernels at the viewer geometry); stftx its round-5 "
                                        "default; fast the opt-in tolerance kernel")
    if rank == 0:
        print(json.dumps(out), flush=True)


def end_to_end(args, plan, kind):
    """PCIe-inclusive rate of the C4 path (H2D int16 + D2H), reported beside the
    value, never as it: a sample of the shard's geometry as int16 PCM (the WAV encoding, 2 B per
    sample) in page-locked host memory -> device -> the same fused kernel (s16 input) -> rows
    back into page-locked host memory, timed over 3 passes after one warm pass."""
    import ctypes as C
    import numpy as np
    from thesia import engine
    from thesia._lib import lib, check
    n_tr = min(100, args.tracks)
    n_samples = int(round(args.seconds * args.sr))
    host = np.empty(n_tr * n_samples * args.channels, np.int16)
    for t in range(n_tr):
        host[t * n_samples * args.channels:(t + 1) * n_samples * args.channels] = \
            engine.synth_pcm_host(args.channels, t, n_samples, args.sr).reshape(-1)
    offs = np.arange(n_tr, dtype=np.uint64) * (n_samples * args.channels)
    lens = np.full(n_tr, n_samples, np.uint64)
    frames = engine.Batch.frames_for(plan, lens)
    out = np.empty(frames * plan.row_bins * (8 if kind == engine.OUT_COMPLEX else 4), np.uint8)
    for a in (host, out):
        check(lib.thesia_host_register(a.ctypes.data_as(C.c_void_p), a.nbytes))
    din = engine.DeviceBuffer(host.nbytes)
    dout = engine.DeviceBuffer(out.nbytes)
    b = engine.Batch(plan, din, offs, lens, dout, input_format=engine.IN_S16, channels=args.channels)

    def one():
        check(lib.thesia_memcpy_h2d(din.ptr, host.ctypes.data_as(C.c_void_p), host.nbytes))
        b.run()
        check(lib.thesia_memcpy_d2h(out.ctypes.data_as(C.c_void_p), dout.ptr, out.nbytes))

    one()
    engine.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        one()
    engine.synchronize()
    dt = (time.perf_counter() - t0) / 3
    b.close()
    for a in (host, out):
        lib.thesia_host_unregister(a.ctypes.data_as(C.c_void_p))
    return {"frames_per_s": frames / dt, "ms_per_pass": dt * 1e3, "frames": frames,
            "h2d_bytes": host.nbytes, "d2h_bytes": out.nbytes,
            "sample": f"{n_tr} tracks of the shard geometry, int16 PCM in page-locked host memory "
                      f"(H2D {host.nbytes / 1e9:.2f} GB + kernel + D2H {out.nbytes / 1e9:.2f} GB)"}


def main_worker(args):
    ws, rank, local, pg = dist_setup()
    if args.selftest:
        main_selftest(args, ws, rank, pg)
        if pg is not None:
            pg.destroy_process_group()
        return
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "multi-spectrogram-viewer_amd"))
    from thesia import engine, shard

    # one rank per GPU; on a box with fewer GPUs than ranks (a rehearsal) ranks share devices
    device = local % max(1, engine.device_count())
    engine.set_device(device)
    if args.workload == "viewer":
        main_viewer(args, rank)
        if pg is not None:
            pg.destroy_process_group()
        return
    if args.workload == "c5":
        main_c5(args, ws, rank, pg, device)
        if pg is not None:
            pg.destroy_process_group()
        return
    n_samples = int(round(args.seconds * args.sr))
    kind = {"mel_db": engine.OUT_MEL_AMP_DB, "amp_db": engine.OUT_AMP_DB,
            "power_db": engine.OUT_POWER_DB, "complex": engine.OUT_COMPLEX}[args.output]
    fmt = engine.IN_F32 if args.input == "f32" else engine.IN_S16
    plan = engine.Plan(args.n_fft, args.win, args.hop, kind, sr=args.sr,
                       n_mels=args.n_mels if kind == engine.OUT_MEL_AMP_DB else 0)
    el = 4 if fmt == engine.IN_F32 else 2
    per_track = n_samples * args.channels
    # the job's tracks (tracks-per-GPU x ranks) are partitioned per file by LPT
    # (thesia.shard); every rank computes the same partition, no exchange
    mine = shard.plan_shards([n_samples] * (args.tracks * ws), args.win, args.hop, args.n_fft,
                             args.n_mels if kind == engine.OUT_MEL_AMP_DB else 0, ws, rank)
    n_local = len(mine)
    din = engine.DeviceBuffer(n_local * per_track * el)
    # distinct tracks per rank: the generator is seeded per rank and track
    engine.synth_pcm_device(din, fmt, args.channels, n_local, n_samples, args.sr, seed=rank)
    offs = np.arange(n_local, dtype=np.uint64) * per_track
    lens = np.full(n_local, n_samples, np.uint64)
    frames = engine.Batch.frames_for(plan, lens)
    dout = engine.DeviceBuffer(frames * plan.row_bins * (8 if kind == engine.OUT_COMPLEX else 4))
    batch = engine.Batch(plan, din, offs, lens, dout, input_format=fmt, channels=args.channels,
                         kernel=args.kernel, row_store=args.row_store if kind == engine.OUT_COMPLEX else 0)
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

    if args.kernels:
        ks = [int(v) for v in args.kernels.split(",")]
        res = {k: [] for k in ks}
        for _ in range(5):  # interleaved rounds
            for k in ks:
                batch.set_option(engine.OPT_KERNEL, k)
                batch.run_timed(1)
                res[k].append(batch.run_timed(3) / 3)
        batch.set_option(engine.OPT_KERNEL, args.kernel)
        if rank == 0:
            print(json.dumps({"kernels_ms": {str(k): {"median": float(np.median(t)), "min": float(min(t))}
                                             for k, t in res.items()}}), flush=True)

    if args.max_blocks:
        ms = [int(v) for v in args.max_blocks.split(",")]
        res = {m: [] for m in ms}
        for _ in range(5):  # interleaved rounds
            for m in ms:
                batch.set_option(engine.OPT_MAX_BLOCKS, m)
                batch.run_timed(1)
                res[m].append(batch.run_timed(3) / 3)
        batch.set_option(engine.OPT_MAX_BLOCKS, 0)
        if rank == 0:
            print(json.dumps({"max_blocks_ms": {str(m): {"median": float(np.median(t)), "min": float(min(t))}
                                                for m, t in res.items()}}), flush=True)

    if args.mel_paths:
        ps = [int(v) for v in args.mel_paths.split(",")]
        res = {q: [] for q in ps}
        for _ in range(5):  # interleaved rounds
            for q in ps:
                batch.set_option(engine.OPT_MEL_PATH, q)
                batch.run_timed(1)
                res[q].append(batch.run_timed(3) / 3)
        batch.set_option(engine.OPT_MEL_PATH, 0)
        if rank == 0:
            print(json.dumps({"mel_paths_ms": {str(q): {"median": float(np.median(t)), "min": float(min(t))}
                                               for q, t in res.items()}}), flush=True)

    # kernel duration from HIP events on the launch stream (roofline numerator / denominator)
    kms = batch.run_timed(max(args.steps, 5)) / max(args.steps, 5)
    kms = max_over_ranks(pg, kms)
    abytes = algorithmic_bytes(args, n_local, n_samples, frames, plan.row_bins)
    achieved = abytes / (kms * 1e-3) / 1e9

    reps = gather_reports(pg, {"device": device, "frames": frames, "tracks": n_local})
    summ = ranks_summary(reps)
    result = {
        "metric": METRIC,
        "value": summ["total_frames"] / dt,
        "unit": "frames/s",
        "n_gpus": summ["n_devices"],
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
                        f"({args.input} interleaved), n_fft {args.n_fft} "
                        f"{'' if args.win == args.n_fft else 'win ' + str(args.win) + ' '}hop {args.hop} Hann, "
                        f"sum-downmix, {'mel-' + str(args.n_mels) + ' + amp dB' if kind == engine.OUT_MEL_AMP_DB else args.output}",
            "tracks_per_gpu": n_local,
            "tracks_total": args.tracks * ws,
            "frames_per_gpu": frames,
            "ranks": ws,
            "devices": summ["devices"],
            "per_rank_frames": summ["per_rank_frames"],
            "parallelism": f"file-sharded x{ws}, no collective",
        },
    }
    if rank == 0:
        rec = profile_record(workload_params(args, batch.kernel))
        result["roofline"] = {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": rec.get("hbm_bytes_per_launch") if rec else None,
            "traffic_source": provenance(rec) if rec else "no stored PMC record of this exact workload",
            "kernel": kernel_name(batch.kernel, args.n_fft)
                      + ": downmix+frame+window+rFFT+" + {"mel_db": "|X|+mel+dB", "amp_db": "|X|+dB",
                                                           "power_db": "|X|^2+dB", "complex": "complex out"}[args.output]
                      + ", one launch",
            "kernel_ms": kms,
            "algorithmic_bytes_per_launch": abytes,
        }
        if kind == engine.OUT_COMPLEX:
            if args.row_stores:
                result["roofline"]["row_stores_ms"] = ab_row_stores(args, batch)
            result["roofline"].update(hbm_ceiling(din, n_local * per_track * el, dout, frames * plan.row_bins * 8))
            result["roofline"]["frac_of_ceiling"] = achieved / result["roofline"]["ceiling_gbs"]
        ic = issue_ceiling(rec, kms) if batch.kernel == 5 else None
        if ic is not None:
            result["roofline_valu_issue"] = ic
        if kind != engine.OUT_COMPLEX and not args.no_rfft_roofline:
            result["roofline_window_rfft"] = rfft_roofline(args, din, offs, lens, fmt, n_local, n_samples)
        if ws == 1 and args.kernel == 0 and not args.no_exact:
            # the same launch on the reference-order streaming kernel (rows equal the oracle's bit
            # for bit, tests/test_gpu_stftr.py / test_gpu_stftq.py), reported beside the line
            try:
                batch.set_option(engine.OPT_KERNEL, 7)
                batch.run_timed(1)
                ems = batch.run_timed(max(3, args.steps // 2)) / max(3, args.steps // 2)
                result["bit_exact"] = {"kernel": kernel_name(7, args.n_fft), "kernel_ms": ems,
                                       "frames_per_s": frames / (ems * 1e-3),
                                       "roofline_frac": abytes / (ems * 1e-3) / 1e9 / HBM_PEAK_GBS}
                batch.set_option(engine.OPT_KERNEL, 0)
            except Exception as e:  # (a geometry kernel 7 does not cover)
                result["bit_exact"] = {"unsupported": str(e)}
        if ws == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args, n_samples)
        if ws == 1 and not args.no_c1:
            result["c1"] = c1_line(args)
        if ws == 1 and not args.no_e2e:
            result["end_to_end_pcie"] = end_to_end(args, plan, kind)
        print(json.dumps(result), flush=True)
    batch.close()
    if pg is not None:
        pg.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus))
    main_worker(args)


if __name__ == "__main__":
    main()
