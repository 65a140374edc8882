#!/usr/bin/env python3
"""Benchmark of the MI355X BCn block-compression hot path.

Metric (BASELINE.json): Mpixels/s (and blocks/s) BC1 & BC7 on 8K RGBA8 at
1/2/4/8 MI355X.

--workload 8k (default) = configs[1]: BC1 default quality on ONE 8192x8192
synthetic RGBA8 texture (G1: gradient + noise), inputs resident in HBM, one
rank per GPU.  With N ranks the texture's 2048 block rows are split over the
ranks (rank r takes shard.shard_rows(2048, N, r): 2048/N contiguous rows) and
a step is the rank's encode of its rows followed by ONE gather of the packed
bitstream to rank 0 (RCCL over xGMI; north_star) -- strong
scaling, the job fixed at one 8K image.  `value` counts that whole step;
`value_kernel_only` the encode alone (the slowest rank's HIP-event time).
--weak gives every rank its own 8192^2 texture instead (weak scaling).  The
same line carries, on the same split: configs[2] legs (BC4 R8 height map,
BC5 RG8 normal map), the fast BC7 path (bc7enc16), BC6H, the configs[4]
batch legs, and configs[3] legs (BC7 default quality over the 8K texture,
one pass each: exact search last, so the driver's tail of the line keeps it).

--workload batch64 = configs[4]: BC7 over a fixed 64 x 4096^2 G1 stack, every
slice's block rows split over the N ranks (strong scaling; chunks of
--shard-chunk block rows dealt round-robin), one timed RCCL gather of the
packed bitstream to rank 0 at the end.

--gpus N without torchrun's environment starts N ranks itself (a
torch.distributed.run child process, before any GPU call); under torchrun
--gpus must equal WORLD_SIZE.

roofline: the encoder's algorithmic bytes (72 B/block BC1,
80 B/block BC7, 24 B/block BC4, 48 B/block BC5) per launch / its average
duration, measured with HIP events on the launch stream, against 8 TB/s; the
binding figure is VALU issue (`roofline.valu`: wave-instructions per launch
from the committed rocprofv3 --pmc summaries under profiles/ over this run's
launch time).  cpu_baseline: the CPU restatement (oracle/, test
infrastructure) timed on a bounded sample of the same texture on the host
cores (rank 0 only); the GPU output of the sampled blocks (after the gather)
is checked against it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FMTS = {"bc1": 1, "bc4": 4, "bc5": 5, "bc7": 7}
ALG_BYTES = {1: 72, 4: 24, 5: 48, 7: 80}   # source texels read + block written
CHANNELS = {1: 4, 4: 1, 5: 2, 7: 4}
HBM_PEAK_GBS = 8000.0                        # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK = 256 * 4 * 2.4e9 / 2              # wave64 VALU instructions/s: 256 CUs x 4 SIMDs, one per 2 cycles
G1_SEED = 0x9E3779B9


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--format", default="bc1", choices=sorted(FMTS))
    p.add_argument("--size", type=int, default=8192, help="texture width = height")
    p.add_argument("--rows", type=int, default=0, help="--format bc7: block rows of the texture to encode (0 = all)")
    p.add_argument("--weak", action="store_true",
                   help="8k workload: every rank encodes its own size^2 texture (weak scaling) instead of its "
                        "block rows of one texture (strong scaling, the default)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--traffic-json", default="")
    p.add_argument("--bc7-quality", type=float, default=1.0,
                   help="BC7BlockEncoder quality for BC7 runs (reference image API: 1.0)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl (= RCCL, the real multi-GPU path) or gloo (rehearsal with ranks sharing a GPU)")
    p.add_argument("--bc7-rows", type=int, default=-1,
                   help="with the default BC1 workload, also time BC7 on this many block rows of the same "
                        "texture (-1 = the whole 8K texture, 0 = skip)")
    p.add_argument("--no-bc45", action="store_true", help="skip the BC4/BC5 8K legs (configs[2])")
    p.add_argument("--bc7-mse-bound", type=float, default=0.5,
                   help="BC7 bounded-exit legs: per-block MSE under which the probe's block is final (0 = no legs); "
                        "the batch64 workload uses this value too (0 = no exit)")
    p.add_argument("--no-bc7enc", action="store_true", help="skip the bc7enc16 (fast BC7 path) legs")
    p.add_argument("--no-g2", action="store_true", help="skip the bounded-exit leg on the G2 texture")
    p.add_argument("--no-host-api", action="store_true",
                   help="skip the host-image (Image_Compress*) end-to-end leg (N = 1 only)")
    p.add_argument("--bc6h-size", type=int, default=1024,
                   help="BC6H leg: HDR float32 texture width = height (0 = skip the leg)")
    p.add_argument("--bc7-shake-ranks", type=int, default=None,
                   help="pruned BC7 search: partitions shaken per single-index mode (gic_options."
                        "bc7_shake_ranks).  8k workload: the pruned legs (default 2; 0 = skip them; the exact "
                        "search is always timed).  batch64: the survivors' search (default 0 = exact, so with "
                        "the bounded exit every block meets the MSE contract by construction)")
    p.add_argument("--workload", default="8k", choices=["8k", "batch64"],
                   help="8k: configs[1] (+ configs[2]/[3] legs); batch64: configs[4], BC7 over a fixed stack "
                        "of --batch-slices x --batch-size^2 G1 slices, block rows of every slice split over "
                        "the ranks (strong scaling) and one timed RCCL gather to rank 0")
    p.add_argument("--batch-slices", type=int, default=64)
    p.add_argument("--batch-size", type=int, default=4096)
    p.add_argument("--no-batch", action="store_true",
                   help="8k workload: skip the configs[4] legs (64 x 4096^2 BC7 batch: bounded exit and exact search)")
    p.add_argument("--no-batch-exact", action="store_true", help="8k workload: skip the exact-search configs[4] leg")
    p.add_argument("--shard-chunk", type=int, default=16,
                   help="batch64: block rows per chunk dealt round-robin over the ranks (0 = one contiguous "
                        "range per rank)")
    a = p.parse_args()
    if a.bc7_shake_ranks is None:
        a.bc7_shake_ranks = 0 if a.workload == "batch64" else 2
    return a


def cpu_model():
    """The host CPU model (BASELINE.md plan)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def relaunch_if_needed(args):
    """--gpus N > 1 without a torchrun environment: start N ranks with
    torch.distributed.run as a CHILD process (before this process touches the
    GPU; no exec) and return its exit code.  None = run in this process."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus <= 1:
            return None
        import socket
        import subprocess
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.call(cmd)
    if int(world_env) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; they must agree")
    return None


def _cpu_threads():
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    return max(1, min(threads, os.cpu_count() or 1, 64))


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    return oracle_lib


# ---------------------------------------------------------------------------
# the split of the 8K workload over the ranks, and the gather to rank 0
# ---------------------------------------------------------------------------

class Split:
    """Block rows of one texture per rank.  Strong (default): rank r takes
    shard.shard_rows(BY, N, r) of the one texture (every rank holds the same
    seeded source in HBM; only its rows are read).  Weak (--weak): every rank
    encodes the whole of its own texture (seed + rank)."""

    def __init__(self, by, world, rank, weak):
        from gfx_imagecompress_amd import shard
        self.by, self.world, self.rank, self.weak = by, world, rank, weak
        if weak or world == 1:
            self.spans = [(0, by)] * world
        else:
            self.spans = [shard.shard_rows(by, world, r) for r in range(world)]
        self.first, self.rows = self.spans[rank]
        self.most = max(n for _, n in self.spans)

    def seed_offset(self):
        return self.rank if self.weak else 0

    def describe(self):
        if self.world == 1:
            return "one rank"
        if self.weak:
            return f"weak scaling: each of {self.world} ranks encodes its own texture"
        return (f"strong scaling: the texture's {self.by} block rows split over {self.world} ranks "
                f"({self.most} contiguous rows each), one gather of the packed blocks to rank 0 per step")


class RootGather:
    """The rank's encode target (padded to the largest shard) and one gather of
    it to rank 0 per step -- torch.distributed.gather into preallocated views of
    one buffer: RCCL's grouped send/recv over xGMI on device tensors, gloo on
    host copies in the rehearsal.  With contiguous equal shards the root's
    buffer is already the image in reference block order.

    Two encode targets alternate over the steps and each gather is issued
    asynchronously, so step k + 1's encode overlaps step k's gather: before an
    encode writes a target, `local` waits for the gather that last read it
    (RCCL: the encode stream waits on the collective, the host does not), and
    drain() waits for the rest before the timed region's closing sync."""

    def __init__(self, split, bx, bb, dev):
        import torch
        import torch.distributed as dist
        self.split, self.bx, self.bb = split, bx, bb
        self.world = split.world
        self.gloo = self.world > 1 and dist.get_backend() == "gloo"
        self.n = split.most * bx * bb
        nbuf = 2 if self.world > 1 else 1
        self.bufs = [torch.empty(max(1, self.n), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
        self.pending = [None] * nbuf
        self.k = 0      # the target the next encode writes
        self.last = 0   # the target the last encode wrote
        self.parts = None
        if self.world > 1 and split.rank == 0:
            buf = torch.empty(self.world * self.n, dtype=torch.uint8, device="cpu" if self.gloo else dev)
            self.parts = list(buf.view(self.world, self.n))

    @property
    def local(self):
        """The encode target of this step (after the gather that last read it)."""
        w = self.pending[self.k]
        if w is not None:
            w.wait()
            self.pending[self.k] = None
        return self.bufs[self.k]

    def __call__(self):
        import torch.distributed as dist
        if self.world <= 1:
            return
        t = self.bufs[self.k].cpu() if self.gloo else self.bufs[self.k]
        self.pending[self.k] = dist.gather(t, gather_list=self.parts, dst=0, async_op=True)
        self.last = self.k
        self.k ^= 1

    def drain(self):
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None

    def tail(self):
        """The per-step gather (None for one rank)."""
        return None if self.world <= 1 else self

    def image_host(self):
        """Rank 0: the blocks of its texture in reference order as a host
        array (strong: the whole gathered image; weak / one rank: its own)."""
        import torch
        self.drain()
        rb = self.bx * self.bb
        if self.world == 1 or self.split.weak:
            return self.bufs[self.last][: self.split.rows * rb].cpu().numpy()
        return torch.cat([self.parts[r][: n * rb] for r, (_, n) in enumerate(self.split.spans)]).cpu().numpy()


def _max_over_ranks(t, world):
    """All-reduce MAX of a small float64 tensor (RCCL on the device, or on the
    host for the gloo rehearsal)."""
    import torch.distributed as dist
    if world <= 1:
        return t
    if dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX)
        return h
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def _gather_root(dst, world):
    """One gather of every rank's (equal-size) packed blocks to rank 0 (RCCL
    on device tensors, gloo on host ones); the concatenation on rank 0, None
    elsewhere."""
    import torch
    import torch.distributed as dist
    gloo = dist.get_backend() == "gloo"
    loc = dst.cpu() if gloo else dst
    parts = [torch.empty_like(loc) for _ in range(world)] if dist.get_rank() == 0 else None
    dist.gather(loc, gather_list=parts, dst=0)
    return torch.cat(parts) if parts is not None else None


def _spread_over_ranks(v, world):
    """[min, max] over ranks of one float (per-rank kernel time: the load
    balance of the shards)."""
    import torch
    import torch.distributed as dist
    if world <= 1:
        return [float(v), float(v)]
    gloo = dist.get_backend() == "gloo"
    dev = "cpu" if gloo else torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([float(v), -float(v)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [-float(t[1]), float(t[0])]


def _timed(world, dev, stream, fn, steps, tail=None):
    """Barrier + sync on both sides of `steps` x (fn(); tail()); returns
    (max-over-ranks wall s of the whole loop, max-over-ranks HIP-event ms per
    fn() on `stream`).  _timed.spread = [min, max] over ranks of the event ms."""
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        fn()
        e1.record(stream)
        if tail is not None:
            tail()
    if tail is not None and hasattr(tail, "drain"):
        tail.drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    own = sum(e0.elapsed_time(e1) for e0, e1 in evs) / steps
    t = _max_over_ranks(torch.tensor([wall, own], dtype=torch.float64, device=dev), world)
    _timed.spread = _spread_over_ranks(own, world)
    return float(t[0]), float(t[1])


def _rates(split, width, px_rows, steps, wall, kern_ms, nd=3):
    """value / value_kernel_only / ms fields of a leg: pixels of the whole job
    (all ranks) per step over the job's wall time, and over the slowest rank's
    encode (HIP events) alone."""
    px = width * (px_rows * split.world if split.weak else px_rows)
    r = {"value": round(px * steps / wall / 1e6, nd), "unit": "Mpixels/s",
         "blocks_per_s": round(px / 16 * steps / wall, 1), "ms_per_step": round(wall / steps * 1e3, 4),
         "kernel_ms": round(kern_ms, 4), "kernel_ms_rank_min_max": [round(x, 4) for x in _timed.spread]}
    if split.world > 1:
        r["value_kernel_only"] = round(px / (kern_ms * 1e-3) / 1e6, nd)
        r["gather_ms_per_step"] = round(max(0.0, wall / steps * 1e3 - kern_ms), 4)
    return r


def _hbm_roofline(fmt_bytes, blocks, kern_ms, traffic=None, bound="valu"):
    alg = fmt_bytes * blocks
    ach = alg / (kern_ms * 1e-3) / 1e9
    return {"bound": bound, "achieved": round(ach, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 8), "traffic": traffic, "alg_bytes_per_launch": alg}


def _valu_roofline(name, size, rows, kern_ms, launch_key=None, scale=1.0):
    """VALU issue roofline of a kernel: SQ_INSTS_VALU per launch from the
    committed PMC summary profiles/<name> (tools/valu_json.py, same workload)
    over this run's measured launch duration (`scale`: the fraction of that
    workload one launch of this run covers, for a rank's share of the
    texture); None when absent or for another workload size."""
    vj = os.path.join(ROOT, "profiles", name)
    try:
        with open(vj) as f:
            vr = json.load(f)
        if vr.get("size") != size or vr.get("rows") != rows:
            return None
        insts = (vr["valu_insts_per_launch"] if launch_key is None else vr[launch_key]) * scale
        rate = insts / (kern_ms * 1e-3)
        return {"achieved": round(rate / 1e12, 4), "peak": round(VALU_PEAK / 1e12, 4),
                "unit": "T wave-instr/s", "frac": round(rate / VALU_PEAK, 4), "insts_per_launch": round(insts),
                "source": os.path.relpath(vj, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def _dominant_kernel(name):
    """The committed per-kernel figures of the dominant kernel of a BC7 pass
    (its own rocprofv3 launch time and SQ_INSTS_VALU)."""
    vj = os.path.join(ROOT, "profiles", name)
    try:
        with open(vj) as f:
            vr = json.load(f)
        k = vr.get("kernel", "")
        k = k[k.find("k_"):k.find("(")] if "k_" in k else k[:40]
        return {"kernel": k, "valu_frac": round(vr["valu_frac"], 4), "launch_ms": round(vr["launch_ms"], 3),
                "insts_per_launch": round(vr["valu_insts_per_launch"]), "source": os.path.relpath(vj, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


# ---------------------------------------------------------------------------
# legs
# ---------------------------------------------------------------------------

def make_source(fmt, size, seed_offset, device):
    import torch
    from gfx_imagecompress_amd import synth
    if fmt in (1, 7):
        return synth.g1_torch(size, size, 1, seed=G1_SEED + seed_offset, device=device)
    h = synth.height_field(size, size, seed=1 + seed_offset)
    if fmt == 4:
        return torch.from_numpy(h[None, :, :, None].copy()).to(device)
    return torch.from_numpy(synth.normal_map(h)[None].copy()).to(device)


def cpu_baseline_rows(fmt, host, size, got_blocks, budget_s, by):
    """Oracle on a bounded prefix of block rows (all threads, a pool over
    block rows); returns (cpu_baseline dict, mismatching blocks)."""
    import numpy as np
    orc = _oracle()
    threads = _cpu_threads()
    bx = (size + 3) // 4
    bb = 8 if fmt in (1, 4) else 16
    rows = min(by, 16)

    def run(n):
        return orc.encode_image(fmt, host, bc4_channel=0, first_row=0, num_rows=n, threads=threads)
    t0 = time.perf_counter()
    out = run(rows)
    dt = time.perf_counter() - t0
    if dt < budget_s / 4 and rows < by:    # grow the sample to ~budget_s of CPU work, bounded by the image
        rows = max(rows, min(by, int(rows * budget_s / max(dt, 1e-3))))
        t0 = time.perf_counter()
        out = run(rows)
        dt = time.perf_counter() - t0
    got = got_blocks.reshape(-1, bb)[: rows * bx]
    mism = int((got != out).any(axis=1).sum())
    res = {"value": round(rows * 4 * size / dt / 1e6, 4), "unit": "Mpixels/s", "cores": threads, "kind": "port",
           "sample": f"block rows 0-{rows - 1} ({rows * bx} blocks, {dt:.2f} s, {threads} threads)",
           "blocks_per_s": round(rows * bx / dt, 1)}
    return res, mism


def bc7_cpu_sample(args, host, size, by, budget_s):
    """The exact BC7 oracle on block rows spread over the texture: row 0, then
    evenly spaced rows until ~budget_s of CPU work (the oracle's pool splits a
    row into 16-block jobs, so every thread is busy), plus a one-thread run
    of 16 blocks to show the pool's per-thread rate.  Returns
    ({row: blocks}, cpu_baseline dict)."""
    orc = _oracle()
    threads = _cpu_threads()
    bx = (size + 3) // 4
    c0 = time.perf_counter()
    one = orc.encode_image_bc7(host[0:4, 0:64], quality=args.bc7_quality, first_row=0, num_rows=1, threads=1)
    dt1 = time.perf_counter() - c0
    rows = {}
    c0 = time.perf_counter()
    rows[0] = orc.encode_image_bc7(host, quality=args.bc7_quality, first_row=0, num_rows=1, threads=threads)
    dt = time.perf_counter() - c0
    more = max(0, min(by - 1, int(budget_s / max(dt, 1e-3)) - 1, 31))
    for i in range(more):
        r = (by * (i + 1)) // (more + 1)
        if r in rows:
            continue
        c0 = time.perf_counter()
        rows[r] = orc.encode_image_bc7(host, quality=args.bc7_quality, first_row=r, num_rows=1, threads=threads)
        dt += time.perf_counter() - c0
    assert (one == rows[0][:16]).all(), "oracle: one-thread and pooled runs differ"
    nb = len(rows) * bx
    bps, bps1 = nb / dt, 16 / dt1
    cpu = {"value": round(len(rows) * 4 * size / dt / 1e6, 6), "unit": "Mpixels/s", "cores": threads, "kind": "port",
           "sample": f"{len(rows)} block rows spread over the texture ({nb} blocks, {dt:.1f} s, {threads} threads "
                     f"on 16-block jobs)",
           "blocks_per_s": round(bps, 1), "blocks_per_s_one_thread": round(bps1, 1),
           "pool_per_thread_vs_one_thread": round(bps / threads / bps1, 3)}
    return rows, cpu


def bc7_leg(args, gic, src, size, split, dev, rank, shake_ranks=0, bound=0.0, ref=None, leg_name=None):
    """configs[3]: BC7 default quality (BC7BlockEncoder quality 1) on the 8K
    texture, one timed pass over the rank's block rows followed by the gather;
    the exact search (`ref` None) also times the CPU restatement on rows spread
    over the texture (rank 0) and checks them bit for bit; the pruned / bounded
    searches are checked on the same rows against the exact oracle's blocks
    under the per-block MSE contract of SURVEY.md 8(d)."""
    import numpy as np
    bx, by = (size + 3) // 4, (size + 3) // 4
    if args.bc7_rows >= 0:      # a band of the texture's first block rows, split over the ranks the same way
        split = Split(min(args.bc7_rows, by), split.world, split.rank, split.weak)
    g = RootGather(split, bx, 16, dev)
    stream = _stream(dev)
    opts = gic.Options(bc7_quality=args.bc7_quality, bc7_shake_ranks=shake_ranks, bc7_mse_bound=bound)
    gic.encode_device(7, src, size, size, 1, 4, g.local, opts, split.first, min(split.rows, 4), stream=stream)

    def enc():
        gic.encode_device(7, src, size, size, 1, 4, g.local, opts, split.first, split.rows, stream=stream)
    gic.iter_cap_hits(reset=True)
    wall, kern_ms = _timed(split.world, dev, stream, enc, 1, tail=g.tail())
    stages = gic.last_bc7_stages()
    hits = gic.iter_cap_hits(reset=True)
    res = _rates(split, size, split.by * 4, 1, wall, kern_ms, nd=4)
    if bound > 0 and len(stages) > 1:
        res["stage_blocks"] = stages
        res["probe_exit_share"] = round(1.0 - stages[-1] / max(stages[0], 1), 4)
    res["ms_per_pass"] = res.pop("ms_per_step")
    res["iter_cap_hits"] = hits
    blocks = split.rows * bx
    res["roofline"] = _hbm_roofline(80, blocks, kern_ms)
    leg = leg_name or ("bc7" if not shake_ranks and not bound else
                       ("bc7_pruned" if not bound else ("bc7_bounded" if not shake_ranks else "bc7_bounded_pruned")))
    valu = _valu_roofline(f"valu_{leg}_pass.json", size, by, kern_ms, launch_key="valu_insts_per_pass",
                          scale=split.rows / by)
    if valu is not None:
        res["roofline"]["valu"] = valu
    dom = _dominant_kernel("valu_bc7_shake8.json") if leg in ("bc7", "bc7_pruned") else None
    if dom is not None:
        res["roofline"]["valu_dominant"] = dom
    if rank == 0 and not args.no_cpu:
        host = src[0].cpu().numpy()
        got = g.image_host().reshape(-1, bx, 16)
        if ref is None:
            rows, cpu = bc7_cpu_sample(args, host, size, split.by, args.cpu_seconds)
            same = sum(int((got[r] == b).all(axis=1).sum()) for r, b in rows.items())
            res["cpu_baseline"] = cpu
            res["gpu_parity"] = f"{same}/{len(rows) * bx} sampled blocks bit-identical to the oracle"
            res["_ref"] = rows
        else:
            orc = _oracle()
            same = bad = 0
            mg_sum = mc_sum = 0.0
            hit = 0
            for r, b in ref.items():
                t = host[4 * r:4 * r + 4, :bx * 4].reshape(4, bx, 4, 4).transpose(1, 0, 2, 3).reshape(bx, 16, 4)
                t = t.astype(np.float64)
                mg = ((orc.bc7_decode(got[r]).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
                mc = ((orc.bc7_decode(b).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
                same += int((got[r] == b).all(axis=1).sum())
                bad += int((mg > mc * 1.001 + 0.5).sum())
                hit += int((mg <= bound).sum())
                mg_sum += float(mg.sum())
                mc_sum += float(mc.sum())
            n = len(ref) * bx
            res["gpu_parity"] = (f"{same}/{n} sampled blocks bit-identical to the exact oracle, {bad} outside the "
                                 f"MSE contract, mean MSE {mg_sum / n:.4f} vs {mc_sum / n:.4f}" +
                                 (f", {hit} within the exit bound" if bound > 0 else ""))
    return res


def g2_bounded_leg(args, gic, size, split, dev, rank):
    """The bounded exit on a second content: G2 (the same gradient, independent
    noise per channel, synth.g2) instead of G1's grey-axis noise.  Reports the
    share of blocks the probes finish (stage_blocks: blocks entering each stage)
    and checks two exact-oracle rows under the contract."""
    from gfx_imagecompress_amd import synth
    src2 = synth.g2_torch(size, size, device=dev)
    ref = None
    if rank == 0 and not args.no_cpu:
        host2 = src2[0].cpu().numpy()
        orc = _oracle()
        by = args.bc7_rows if args.bc7_rows > 0 else (size + 3) // 4
        ref = {r: orc.encode_image_bc7(host2, quality=args.bc7_quality, first_row=r, num_rows=1,
                                       threads=_cpu_threads()) for r in (0, by // 2)}
    res = bc7_leg(args, gic, src2, size, split, dev, rank, 0, args.bc7_mse_bound, ref=ref,
                  leg_name="bc7_bounded_g2")
    out = dict(metric=f"BC7 q{args.bc7_quality:g}, bounded exit (MSE {args.bc7_mse_bound:g}) + exact survivors, "
                      f"G2 (independent per-channel noise)", **res)
    del src2
    return out


def _stream(dev):
    import torch
    return torch.cuda.current_stream(dev)


def simple_leg(args, gic, fmt, split, dev, rank, src, width, height, channels, enc_fn, steps, warmup,
               oracle_fn=None, sample_rows=16):
    """A leg timed as `steps` x (encode of the rank's rows; gather), plus
    (rank 0) the CPU restatement on a bounded sample of block rows whose GPU
    output, after the gather, is checked bit for bit."""
    import numpy as np
    bx = (width + 3) // 4
    bb = gic.block_bytes(fmt) if fmt != gic.FMT_BC7ENC16 else 16
    g = RootGather(split, bx, bb, dev)
    stream = _stream(dev)

    def enc():
        enc_fn(g.local, split.first, split.rows, stream)
    for _ in range(max(1, warmup)):
        enc()
    wall, kern_ms = _timed(split.world, dev, stream, enc, steps, tail=g.tail())
    res = _rates(split, width, split.by * 4, steps, wall, kern_ms)
    res["_blocks"] = split.rows * bx
    if rank == 0 and not args.no_cpu and oracle_fn is not None:
        threads = _cpu_threads()
        got = g.image_host().reshape(-1, bb)
        rows = min(split.by, sample_rows)
        c0 = time.perf_counter()
        ref = oracle_fn(0, rows, threads)
        dt = time.perf_counter() - c0
        budget = args.cpu_seconds / 2   # grow the sample to ~budget s of CPU work, bounded by the image
        if dt < budget / 4 and rows < split.by:
            rows = int(min(split.by, max(rows, rows * budget / max(dt, 1e-3))))
            c0 = time.perf_counter()
            ref = oracle_fn(0, rows, threads)
            dt = time.perf_counter() - c0
        ref = ref.reshape(-1, bb)
        mism = int((got[: len(ref)] != ref).any(axis=1).sum())
        res["cpu_baseline"] = {"value": round(rows * 4 * width / dt / 1e6, 5), "unit": "Mpixels/s", "cores": threads,
                               "kind": "port", "sample": f"block rows 0-{rows - 1} ({rows * bx} blocks, {dt:.2f} s)",
                               "blocks_per_s": round(rows * bx / dt, 1)}
        res["gpu_parity"] = "bit-exact" if mism == 0 else f"{mism} blocks differ"
    return res


def bc45_leg(args, gic, fmt, split, dev, rank):
    """configs[2]: BC4 on an R8 8192^2 height map (channel 0) or BC5 on its RG8
    normal map, block rows split like the BC1 leg."""
    size = args.size
    src = make_source(fmt, size, split.seed_offset(), dev)
    opts = gic.Options(bc4_channel=0)
    ch = CHANNELS[fmt]
    host = src[0].cpu().numpy() if split.rank == 0 else None

    def enc(dst, first, rows, stream):
        gic.encode_device(fmt, src, size, size, 1, ch, dst, opts, first, rows, stream=stream)

    def orc(first, rows, threads):
        return _oracle().encode_image(fmt, host, bc4_channel=0, first_row=first, num_rows=rows, threads=threads)
    res = simple_leg(args, gic, fmt, split, dev, split.rank, src, size, size, ch, enc, args.steps, args.warmup, orc)
    nb = res.pop("_blocks")
    out = {"metric": f"{'BC4 R8 height' if fmt == 4 else 'BC5 RG8 normal'} {size}x{size}"}
    out.update(res)
    out["roofline"] = _hbm_roofline(ALG_BYTES[fmt], nb, res["kernel_ms"], bound="hbm")
    return out


def bc7enc16_leg(args, gic, src, size, split, dev, fast):
    """The reference's fast BC7 path (bc7enc16, Image_CompressRichGel999BC7,
    richgel999_bc7enc16.cpp:21-71; ImageCompress_Compress(DXBC7, fast=true)) on
    the same 8K G1 texture."""
    opts = gic.Options.bc7enc16(fast=fast, perceptual=True)
    host = src[0].cpu().numpy() if split.rank == 0 else None

    def enc(dst, first, rows, stream):
        gic.encode_device(gic.FMT_BC7ENC16, src, size, size, 1, 4, dst, opts, first, rows, stream=stream)

    def orc(first, rows, threads):
        return _oracle().encode_image_bc7enc_rows(host, first, rows, threads=threads, fast=fast, perceptual=True)
    res = simple_leg(args, gic, gic.FMT_BC7ENC16, split, dev, split.rank, src, size, size, 4, enc, args.steps,
                     args.warmup, orc, sample_rows=4)
    nb = res.pop("_blocks")
    out = {"metric": f"bc7enc16 (fast BC7 path), perceptual, uber {0 if fast else 4}"}
    out.update(res)
    out["roofline"] = _hbm_roofline(80, nb, res["kernel_ms"])
    valu = _valu_roofline("valu_bc7enc16_fast.json" if fast else "valu_bc7enc16.json", size, size, res["kernel_ms"],
                          scale=split.rows / split.by)
    if valu is not None:
        out["roofline"]["valu"] = valu
    return out


def bc6h_leg(args, gic, split_of, dev, rank, signed=False):
    """BC6H (BC6HBlockEncoder at the image API's quality 1.0;
    unsigned half floats, or signed) on a synthetic HDR float32 texture
    (synth.hdr_rgba), block rows split like the other legs, plus (rank 0) the
    CPU restatement on a bounded sample of whole blocks."""
    import numpy as np
    import torch
    from gfx_imagecompress_amd import synth
    n = args.bc6h_size
    bx = by = (n + 3) // 4
    split = split_of(by)
    img = synth.hdr_rgba(n, n, seed=1 + split.seed_offset(), signed=signed)
    src = torch.from_numpy(img.reshape(-1).copy()).to(dev)
    fmt = gic.FMT_BC6H_SF if signed else gic.FMT_BC6H
    g = RootGather(split, bx, 16, dev)
    stream = _stream(dev)

    def enc():
        gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, n, n, 1, 4, g.local, first_block_row=split.first,
                              num_block_rows=split.rows, stream=stream)
    enc()
    steps = max(1, min(args.steps, 3))
    gic.iter_cap_hits(reset=True)
    wall, kern_ms = _timed(split.world, dev, stream, enc, steps, tail=g.tail())
    hits = gic.iter_cap_hits(reset=True)
    res = {"metric": f"BC6H {'signed' if signed else 'unsigned'} {n}x{n} HDR float32"}
    res.update(_rates(split, n, by * 4, steps, wall, kern_ms))
    res.update({"steps": steps, "iter_cap_hits": hits})
    res["roofline"] = _hbm_roofline(272, split.rows * bx, kern_ms)
    valu = _valu_roofline("valu_bc6h_shake_signed.json" if signed else "valu_bc6h_shake.json", n, n, kern_ms,
                          launch_key="valu_insts_per_step", scale=split.rows / by)
    if valu is not None:
        res["roofline"]["valu"] = valu
    if rank == 0 and not args.no_cpu:
        threads = _cpu_threads()
        rows = min(by, 4)
        ys = np.minimum(np.arange(rows * 4), n - 1)
        xs = np.minimum(np.arange(bx * 4), n - 1)
        t = img[ys][:, xs]
        blocks = t.reshape(rows, 4, bx, 4, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 64)
        nsamp = min(len(blocks), 1024)
        c0 = time.perf_counter()
        ref, _ = _oracle().bc6h_blocks(blocks[:nsamp], signed=signed, threads=threads)
        dt = time.perf_counter() - c0
        got = g.image_host().reshape(-1, 16)[:nsamp]
        res["cpu_baseline"] = {"value": round(nsamp * 16 / dt / 1e6, 5), "unit": "Mpixels/s", "cores": threads,
                               "kind": "port", "sample": f"{nsamp} blocks of block rows 0-{rows - 1} ({dt:.2f} s)",
                               "blocks_per_s": round(nsamp / dt, 1)}
        res["gpu_parity"] = "bit-exact" if np.array_equal(got, ref) else \
            f"{int((got != ref).any(axis=1).sum())} blocks differ"
    return res


# ---------------------------------------------------------------------------
# configs[4]: the 64 x 4096^2 batch
# ---------------------------------------------------------------------------

def _batch_check_rows(S, by):
    """(slice, block row) pairs the batch legs check against the oracle: slices
    spread over the stack, the middle row, a shard-chunk boundary row and the
    last row."""
    return sorted({(0, by // 2), (S // 2, max(0, min(by - 1, 16 * (by // 32) - 1))), (S - 1, by - 1)})


def _batch_oracle(args, S, n, bx, by, cache):
    """The exact oracle's blocks of the check rows (computed once per run,
    shared by the exact and the bounded legs; the pool splits each row into
    16-block jobs) and the CPU time they took."""
    if "rows" in cache:
        return cache["rows"], cache["dt"], cache["threads"]
    orc = _oracle()
    from gfx_imagecompress_amd import synth
    threads = _cpu_threads()
    rows, dt = {}, 0.0
    for sl, row in _batch_check_rows(S, by):
        img = synth.g1(n, n, seed=G1_SEED + sl)
        c0 = time.perf_counter()
        rows[(sl, row)] = (orc.encode_image_bc7(img, quality=args.bc7_quality, first_row=row, num_rows=1,
                                                threads=threads), img[4 * row:4 * row + 4, :bx * 4])
        dt += time.perf_counter() - c0
    cache.update(rows=rows, dt=dt, threads=threads)
    return rows, dt, threads


def batch_run(args, gic, world, rank, dev, bound, shake_ranks, steps, warmup, src=None, oracle_cache=None):
    """configs[4]: BC7 (quality 1) over a fixed stack of S G1 slices (slice s
    seeded 0x9E3779B9+s), every slice's block rows split over the ranks
    (strong scaling: the batch is fixed, each rank does 1/N) in chunks of
    --shard-chunk rows dealt round-robin (shard.row_ranges; 0 = contiguous);
    a step = the rank's gic_hip_encode_rows calls (one per range, every slice
    at once).  After the timed steps one gather (RCCL on GPUs) brings every
    shard to rank 0, which restores the reference block order (timed
    separately) and checks block rows of several slices against the oracle:
    bit-identity for the exact search, the per-block MSE contract for the
    bounded exit.  Returns the result dict on rank 0 (None elsewhere)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from gfx_imagecompress_amd import shard, synth
    S, n = args.batch_slices, args.batch_size
    bx = by = (n + 3) // 4
    chunk = args.shard_chunk
    ranges = shard.row_ranges(by, world, rank, chunk)
    nblk = shard.shard_blocks(by, bx, S, world, rank, chunk)
    if src is None:
        src = synth.g1_torch(n, n, S, seed=G1_SEED, device=dev)
    dst = torch.empty(max(1, nblk * 16), dtype=torch.uint8, device=dev)
    opts = gic.Options(bc7_quality=args.bc7_quality, bc7_shake_ranks=shake_ranks, bc7_mse_bound=bound)
    stream = _stream(dev)
    # warm-up: the per-device tables and workspaces (one block row of one slice)
    if ranges:
        gic.encode_device(7, src[:1], n, n, 1, 4, dst, opts, ranges[0][0], 1, stream=stream)

    def step():
        shard.encode_shard(7, src, n, n, S, 4, rank, world, opts, stream=stream, chunk=chunk, dst=dst)
    for _ in range(warmup):
        step()
    gic.iter_cap_hits(reset=True)
    wall, kern_ms = _timed(world, dev, stream, step, steps)
    spread = _timed.spread
    hits = _max_over_ranks(torch.tensor([float(gic.iter_cap_hits(reset=True))], dtype=torch.float64, device=dev),
                           world)
    gather_ms = None
    full = dst
    if world > 1:
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        full = shard.gather_to_root(dst[:nblk * 16], 7, n, n, S, world, chunk=chunk)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) * 1e3
        g = _max_over_ranks(torch.tensor([gather_ms], dtype=torch.float64, device=dev), world)
        gather_ms = float(g[0])
    total_blocks = S * bx * by
    if rank != 0:
        return None
    how = "one contiguous range per rank" if not chunk else f"chunks of {chunk} block rows dealt round-robin"
    if world == 1:
        gather = "one rank: no gather"
    else:
        gather = (f"{'RCCL' if dist.get_backend() != 'gloo' else 'gloo (rehearsal)'} gather to rank 0 "
                  f"timed separately")
    if bound > 0:
        search = (f"bounded exit (MSE {bound:g}) + " +
                  ("exact survivors (contract met by construction)" if shake_ranks == 0 else "pruned survivors"))
    else:
        search = ("exact (the reference search)" if shake_ranks == 0 else
                  f"pruned, {shake_ranks} partitions shaken per mode (per-block MSE tolerance)")
    res = {
        "metric": f"BC7 q{args.bc7_quality:g} configs[4] batch, {search}",
        "value": round(S * n * n * steps / wall / 1e6, 4), "unit": "Mpixels/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(wall / steps * 1e3, 3), "scaling": "strong", "dtype": "f64+int32",
        "config": {"workload": f"configs[4]: BC7 quality {args.bc7_quality:g} on a batch of {S}x{n}x{n} RGBA8 G1 "
                               f"slices (seed 0x9E3779B9+s), block rows of every slice split over {world} rank(s) "
                               f"({how}), {gather}",
                   "format": "BC7", "slices": S, "width": n, "global_batch_blocks": total_blocks,
                   "bc7_search": search, "parallelism": f"block-row shards x{world}", "shard_chunk_rows": chunk},
        "blocks_per_s": round(total_blocks * steps / wall, 1),
        "kernel_ms": round(kern_ms, 3), "kernel_ms_rank_min_max": [round(x, 3) for x in spread],
        "gather_ms": None if gather_ms is None else round(gather_ms, 3),
        "iter_cap_hits": int(hits[0]),
        "roofline": _hbm_roofline(80, nblk, kern_ms),
        "cpu_baseline": None,
    }
    valu = _valu_roofline("valu_batch64_exact_pass.json" if bound == 0 else "valu_batch64_bounded_pass.json",
                          n, by * S, kern_ms, launch_key="valu_insts_per_pass", scale=nblk / total_blocks)
    if valu is not None:
        res["roofline"]["valu"] = valu
    host = full.cpu().numpy().reshape(S, by, bx, 16) if full is not None and \
        full.numel() >= total_blocks * 16 else None
    if not args.no_cpu and host is not None:
        orc = _oracle()
        rows, dt, threads = _batch_oracle(args, S, n, bx, by, oracle_cache if oracle_cache is not None else {})
        same = bad = tot = 0
        mse_g = mse_c = 0.0
        for (sl, row), (ref, texels) in rows.items():
            got = host[sl, row]
            same += int((got == ref).all(axis=1).sum())
            tot += bx
            t = texels.reshape(4, bx, 4, 4).transpose(1, 0, 2, 3).reshape(bx, 16, 4).astype(np.float64)
            mg = ((orc.bc7_decode(got).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
            mc = ((orc.bc7_decode(ref).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
            bad += int((mg > mc * 1.001 + 0.5).sum())
            mse_g += float(mg.sum())
            mse_c += float(mc.sum())
        where = ", ".join(f"s{sl} r{row}" for sl, row in rows)
        res["cpu_baseline"] = {"value": round(len(rows) * 4 * n / dt / 1e6, 6), "unit": "Mpixels/s",
                               "cores": threads, "kind": "port",
                               "sample": f"the exact search on {len(rows)} block rows ({where}; {tot} blocks, "
                                         f"{dt:.1f} s, {threads} threads on 16-block jobs)",
                               "blocks_per_s": round(tot / dt, 1)}
        res["gpu_parity"] = (f"{same}/{tot} blocks{' (after the gather)' if world > 1 else ''} bit-identical to "
                             f"the exact oracle, {bad} outside the MSE contract, mean MSE {mse_g / tot:.4f} vs "
                             f"{mse_c / tot:.4f}")
        res["gpu_parity_ok"] = same == tot if (shake_ranks == 0 and bound == 0) else bad == 0
    return res


def batch_workload(args, gic, world, rank, dev):
    """--workload batch64: configs[4] as the headline line (batch_run)."""
    import torch.distributed as dist
    res = batch_run(args, gic, world, rank, dev, args.bc7_mse_bound, args.bc7_shake_ranks, args.steps, args.warmup)
    if rank == 0:
        line = {"metric": "Mpixels/s (and blocks/s) BC1 & BC7 on 8K RGBA8 at 1/2/4/8 MI355X",
                "value": res["value"], "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": res["ms_per_step"], "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64+int32", "data": "synthetic",
                "config": dict(res["config"], world_size_seen=dist.get_world_size() if world > 1 else 1)}
        for k in ("blocks_per_s", "kernel_ms", "kernel_ms_rank_min_max", "gather_ms", "iter_cap_hits", "roofline",
                  "cpu_baseline", "gpu_parity"):
            line[k] = res.get(k)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# the drop-in host path: host image in, host blocks out (Image_Compress*)
# ---------------------------------------------------------------------------

def host_api_leg(args, gic, src, size, dev, kernel_ms):
    """Image_CompressAMDBC1 (the reference's entry, NULL options) and the BC7
    bounded exit (gic_compress_image) on the 8K host image, end to end: the
    upload of the pageable source, the pipelined encode and the download into
    the returned header.  Beside it the same bytes moved alone (a pageable and a
    pinned 256 MiB upload) and the device-resident kernel time, so the line shows
    how close the pipeline gets to max(upload, kernel)."""
    import numpy as np
    import torch
    host = np.ascontiguousarray(src[0].cpu().numpy())
    mpix = size * size / 1e6

    def timed_copy(t_src, reps=3):
        d = torch.empty(t_src.shape, dtype=t_src.dtype, device=dev)
        best = 1e30
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            d.copy_(t_src)
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t0)
        return best * 1e3

    pageable_ms = timed_copy(torch.from_numpy(host))
    pinned_ms = timed_copy(torch.from_numpy(host).pin_memory())
    want1 = torch.empty((size // 4) * (size // 4) * 8, dtype=torch.uint8, device=dev)
    gic.encode_device(1, src, size, size, 1, 4, want1, gic.Options())
    want1 = want1.cpu().numpy()
    out = {"note": "end to end = host header in -> pipelined upload / encode / download -> host header out; "
                   "pieces of 2^18 blocks (BC7 2^20); GIC_H2D selects the upload mode",
           "upload_alone_ms": {"pageable": round(pageable_ms, 3), "pinned": round(pinned_ms, 3)},
           "bc1_kernel_ms": round(kernel_ms, 4)}
    modes = {}
    old = os.environ.get("GIC_H2D")
    hi = gic.HostImage(host)
    try:
        for mode in ("pageable", "staged", "register"):
            os.environ["GIC_H2D"] = mode
            times, rep_best, ok = [], None, True
            for _ in range(1 + 3):
                got = hi.compress(1, entry="Image_CompressAMDBC1")
                ok = ok and got is not None and np.array_equal(got.reshape(-1), want1)
                rep = gic.host_report()
                times.append(hi.last_call_ms)
                if rep_best is None or rep["total_ms"] < rep_best["total_ms"]:
                    rep_best = rep
            e2e = min(times[1:])
            bound = max(pageable_ms if mode == "pageable" else pinned_ms, kernel_ms)
            modes[mode] = {"e2e_ms": round(e2e, 3), "mpix_s": round(mpix / (e2e / 1e3), 1),
                           "h2d_ms": round(rep_best["h2d_ms"], 3), "encode_ms": round(rep_best["encode_ms"], 3),
                           "d2h_ms": round(rep_best["d2h_ms"], 3), "pieces": rep_best["pieces"],
                           "e2e_over_max_upload_kernel": round(e2e / bound, 3),
                           "bytes_equal_device_path": bool(ok)}
        best = min(modes, key=lambda m: modes[m]["e2e_ms"])
        out["bc1"] = dict(mode=best, **modes[best])
        out["bc1_modes"] = modes
        os.environ["GIC_H2D"] = best
        if args.bc7_rows != 0:
            o = gic.Options(bc7_mse_bound=0.5)
            times = []
            for _ in range(2):
                got7 = hi.compress(7, o)
                times.append(hi.last_call_ms)
            rep = gic.host_report()
            out["bc7_bounded"] = {"mode": best, "e2e_ms": round(min(times), 2),
                                  "mpix_s": round(mpix / (min(times) / 1e3), 1),
                                  "h2d_ms": round(rep["h2d_ms"], 3), "encode_ms": round(rep["encode_ms"], 2),
                                  "d2h_ms": round(rep["d2h_ms"], 3), "pieces": rep["pieces"],
                                  "blocks": int(got7.size // 16)}
    finally:
        hi.close()
        if old is None:
            os.environ.pop("GIC_H2D", None)
        else:
            os.environ["GIC_H2D"] = old
    return out


# ---------------------------------------------------------------------------
# the 8K workload (configs[1]-[3]) and the headline line
# ---------------------------------------------------------------------------

def main():
    args = parse()
    rc = relaunch_if_needed(args)
    if rc is not None:
        sys.exit(rc)
    import torch
    import torch.distributed as dist
    import gfx_imagecompress_amd as gic

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":
        # rehearsal of the N>1 logic with more ranks than GPUs (ranks share devices)
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != world:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    dev = torch.device("cuda", local)
    if args.workload == "batch64":
        return batch_workload(args, gic, world, rank, dev)
    fmt = FMTS[args.format]
    size = args.size
    bx, by = (size + 3) // 4, (size + 3) // 4
    if args.rows:
        by = min(args.rows, by)
    split = Split(by, world, rank, args.weak)
    src = make_source(fmt, size, split.seed_offset(), dev)
    ch = CHANNELS[fmt]
    opts = gic.Options(bc4_channel=0, bc7_quality=args.bc7_quality,
                       bc7_shake_ranks=args.bc7_shake_ranks if fmt == 7 else 0)
    stream = _stream(dev)
    g = RootGather(split, bx, gic.block_bytes(fmt), dev)

    def enc():
        gic.encode_device(fmt, src, size, size, 1, ch, g.local, opts, split.first, split.rows, stream=stream)

    for _ in range(args.warmup):
        enc()
    wall, kern_ms = _timed(world, dev, stream, enc, args.steps, tail=g.tail())
    head = _rates(split, size, by * 4, args.steps, wall, kern_ms)
    nblocks = split.rows * bx
    traffic = None
    tj = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{args.format}.json")
    if os.path.exists(tj):
        try:
            with open(tj) as f:
                tr = json.load(f)
            if tr.get("size") == size and tr.get("rows") == by * 4:
                traffic = round(tr.get("hbm_bytes_per_launch") * split.rows / by)
        except (OSError, ValueError, TypeError):
            traffic = None
    roof = _hbm_roofline(ALG_BYTES[fmt], nblocks, kern_ms, traffic, bound="hbm")
    roof["note"] = "compute (VALU) bound; the HBM fraction per BASELINE.json, the binding VALU issue in .valu"
    valu = _valu_roofline(f"valu_{args.format}.json", size, by * 4, kern_ms, scale=split.rows / by)
    if valu is not None:
        roof["valu"] = valu
    # the headline's CPU baseline and parity: block rows of the gathered image
    cpu = None
    if rank == 0 and not args.no_cpu:
        torch.cuda.synchronize(dev)
        cpu, mism = cpu_baseline_rows(fmt, src[0].cpu().numpy(), size, g.image_host(), args.cpu_seconds, by)
        cpu["cpu_model"] = cpu_model()
        cpu["gpu_parity"] = "bit-exact" if mism == 0 else f"{mism} blocks differ"
    del g

    legs = {}
    if fmt == 1 and world == 1 and not args.no_host_api:
        legs["host_api"] = host_api_leg(args, gic, src, size, dev, head["kernel_ms"])
    if fmt == 1 and not args.no_bc45:
        for f in (4, 5):
            legs[f"bc{f}"] = bc45_leg(args, gic, f, Split(by, world, rank, args.weak), dev, rank)
    if fmt == 1 and args.bc6h_size > 0:
        def split_of(b):
            return Split(b, world, rank, args.weak)
        legs["bc6h"] = bc6h_leg(args, gic, split_of, dev, rank)
        legs["bc6h_signed"] = bc6h_leg(args, gic, split_of, dev, rank, signed=True)
    if fmt == 1 and not args.no_bc7enc:
        legs["bc7enc16"] = bc7enc16_leg(args, gic, src, size, split, dev, fast=False)
        legs["bc7enc16_fast"] = bc7enc16_leg(args, gic, src, size, split, dev, fast=True)
    if fmt == 1 and not args.no_batch:
        # configs[4] at its size: the 64 x 4096^2 G1 stack, one pass each of the
        # bounded exit (exact survivors) and the exact reference search, block
        # rows dealt over the ranks, one gather to rank 0, oracle rows checked
        from gfx_imagecompress_amd import synth
        bsrc = synth.g1_torch(args.batch_size, args.batch_size, args.batch_slices, seed=G1_SEED, device=dev)
        cache = {}
        legs["batch64_bounded"] = batch_run(args, gic, world, rank, dev, args.bc7_mse_bound or 0.5, 0, 1, 0,
                                            src=bsrc, oracle_cache=cache)
        if not args.no_batch_exact:
            legs["batch64_exact"] = batch_run(args, gic, world, rank, dev, 0.0, 0, 1, 0, src=bsrc,
                                              oracle_cache=cache)
        del bsrc
        torch.cuda.empty_cache()
    bc7 = {}
    if fmt == 1 and args.bc7_rows != 0:
        # configs[3]: the exact search first (its oracle rows check the others), printed last
        q = args.bc7_quality
        exact = dict(metric=f"BC7 quality {q:g} (all modes, shakers on), exact reference search",
                     **bc7_leg(args, gic, src, size, split, dev, rank))
        ref = exact.pop("_ref", None)
        if args.bc7_shake_ranks > 0:
            bc7["bc7_pruned"] = dict(metric=f"BC7 q{q:g}, pruned: {args.bc7_shake_ranks} partitions shaken per mode",
                                     **bc7_leg(args, gic, src, size, split, dev, rank, args.bc7_shake_ranks, ref=ref))
        if args.bc7_mse_bound > 0:
            if args.bc7_shake_ranks > 0:
                bc7["bc7_bounded_pruned"] = dict(
                    metric=f"BC7 q{q:g}, bounded exit (MSE {args.bc7_mse_bound:g}) + pruned survivors",
                    **bc7_leg(args, gic, src, size, split, dev, rank, args.bc7_shake_ranks, args.bc7_mse_bound,
                              ref=ref))
            bc7["bc7_bounded"] = dict(
                metric=f"BC7 q{q:g}, bounded exit (MSE {args.bc7_mse_bound:g}) + exact survivors",
                **bc7_leg(args, gic, src, size, split, dev, rank, 0, args.bc7_mse_bound, ref=ref))
            if not args.no_g2:
                bc7["bc7_bounded_g2"] = g2_bounded_leg(args, gic, size, split, dev, rank)
        bc7["bc7"] = exact
    elif fmt == 7 and rank == 0:
        roof["valu_dominant"] = _dominant_kernel("valu_bc7_shake8.json")

    if rank == 0:
        line = {
            "metric": "Mpixels/s (and blocks/s) BC1 & BC7 on 8K RGBA8 at 1/2/4/8 MI355X",
            "value": head["value"],
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak" if (args.weak and world > 1) else "strong",
            "vs_baseline": None,
            "dtype": "f32" if fmt != 7 else "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.format.upper()} default quality on a {size}x{by * 4} synthetic "
                                   f"{'RGBA8 G1 gradient+noise' if fmt in (1, 7) else ('R8 height' if fmt == 4 else 'RG8 normal')}"
                                   f" texture; {split.describe()}",
                       "format": args.format.upper(), "width": size, "rows_per_gpu": split.rows * 4,
                       "global_batch_blocks": nblocks * world if args.weak else bx * by,
                       "parallelism": f"block-row shards x{world}",
                       "world_size_seen": dist.get_world_size() if world > 1 else 1},
        }
        for k in ("value_kernel_only", "gather_ms_per_step", "blocks_per_s", "kernel_ms", "kernel_ms_rank_min_max"):
            if k in head:
                line[k] = head[k]
        line["roofline"] = roof
        line["cpu_baseline"] = cpu
        if world > 1:
            line["multi_gpu_note"] = "gather over RCCL/xGMI timed inside every step"
        line.update(legs)
        line.update(bc7)      # the BC7 8K legs last: the exact search is the line's final key
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
