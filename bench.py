#!/usr/bin/env python3
"""Benchmark of the MI355X BCn block-compression hot path.

Metric (BASELINE.json): Mpixels/s (and blocks/s) BC1 & BC7 on 8K RGBA8.

--workload 8k (default) = configs[1]: BC1 default quality on an 8192x8192
synthetic RGBA8 texture (G1: gradient + noise), inputs resident in HBM, one
rank per GPU.  With N ranks the job is an (8192*N) x 8192 texture sharded by
block rows, each rank encoding its own 8192-row shard (weak scaling, no
collective in the timed region; the optional RCCL gather of the packed
bitstream is timed separately with --gather).  The same line carries a
configs[3] leg (BC7 default quality over the same texture, one pass) and
configs[2] legs (BC4 R8 height map, BC5 RG8 normal map, 8192^2).

--workload batch64 = configs[4]: BC7 over a fixed 64 x 4096^2 G1 stack, every
slice's block rows split over the N ranks (strong scaling; chunks of
--shard-chunk block rows dealt round-robin), one timed RCCL gather of the
packed bitstream to rank 0 at the end.

--gpus N without torchrun's environment starts N ranks itself (a
torch.distributed.run child process, before any GPU call); under torchrun
--gpus must equal WORLD_SIZE.

A "step" = one launch of the encoder over the rank's whole shard.  value =
pixels of all ranks x steps / max-over-ranks wall time.  roofline: the
encoder kernel's algorithmic bytes (72 B/block BC1, 80 B/block
BC7, 24 B/block BC4, 48 B/block BC5) per launch / its average duration,
measured with HIP events on the launch stream, against 8 TB/s.  cpu_baseline:
the CPU restatement (oracle/, test infrastructure) timed on a bounded sample
of block rows of the same texture on the host cores (rank 0 only); the GPU
output of those rows is checked bit-for-bit against it.
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


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--format", default="bc1", choices=sorted(FMTS))
    p.add_argument("--size", type=int, default=8192, help="texture width = rows per rank")
    p.add_argument("--rows", type=int, default=0, help="BC7: block rows per rank (0 = all)")
    p.add_argument("--gather", action="store_true", help="time an RCCL gather of the bitstream to rank 0")
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
    p.add_argument("--bc6h-size", type=int, default=1024,
                   help="BC6H leg: HDR float32 texture width = height per rank (0 = skip the leg)")
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
    """The host CPU model and the threads this process may use (BASELINE.md plan)."""
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


def make_source(fmt, size, rank, device):
    import torch
    from gfx_imagecompress_amd import synth
    if fmt in (1, 7):
        return synth.g1_torch(size, size, 1, seed=0x9E3779B9 + rank, device=device)
    import numpy as np
    h = synth.height_field(size, size, seed=1 + rank)
    if fmt == 4:
        return torch.from_numpy(h[None, :, :, None].copy()).to(device)
    return torch.from_numpy(synth.normal_map(h)[None].copy()).to(device)


def cpu_baseline(fmt, src_host, size, gpu_blocks, budget_s, avail_rows, bc7_quality=1.0):
    """Oracle on a bounded prefix of block rows; returns (dict, parity_ok)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1, 64))
    bx = (size + 3) // 4
    by = min((size + 3) // 4, avail_rows)
    rows = min(by, 2 if fmt == 7 else 16)

    def run(n):
        if fmt == 7:
            return oracle_lib.encode_image_bc7(src_host, quality=bc7_quality, first_row=0, num_rows=n, threads=threads)
        return oracle_lib.encode_image(fmt, src_host, bc4_channel=0, first_row=0, num_rows=n, threads=threads)
    t0 = time.perf_counter()
    out = run(rows)
    dt = time.perf_counter() - t0
    # grow the sample to ~budget_s of CPU work (bounded by the image)
    if dt < budget_s / 4 and rows < by:
        more = int(min(by, max(rows, rows * (budget_s / max(dt, 1e-3)))))
        more = max(rows, min(by, more))
        if more > rows:
            rows = more
            t0 = time.perf_counter()
            out = run(rows)
            dt = time.perf_counter() - t0
    px = rows * 4 * size
    gpu_rows = gpu_blocks.reshape(-1, bx, out.shape[1])[:rows].reshape(out.shape)
    parity = bool(np.array_equal(gpu_rows, out))
    mism = int((gpu_rows != out).any(axis=1).sum())
    res = {"value": round(px / dt / 1e6, 4), "unit": "Mpixels/s", "cores": threads, "kind": "port",
           "sample": f"block rows 0-{rows - 1} of rank 0's {size}x{size} texture ({rows * bx} blocks, "
                     f"{dt:.1f} s, {threads} threads)",
           "blocks_per_s": round(rows * bx / dt, 1)}
    return res, parity, mism


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


def bc7_secondary(args, gic, src, size, avail_rows, world, dev, rank, shake_ranks=0, ref_rows=None, bound=0.0):
    """BC7 default quality (configs[3]) on the same texture: one timed pass over
    `--bc7-rows` block rows per rank after a short warm-up, plus (rank 0) the
    CPU restatement on one block row with a bit-exactness check."""
    import torch
    import torch.distributed as dist
    bx = (size + 3) // 4
    rows = avail_rows if args.bc7_rows < 0 else min(args.bc7_rows, avail_rows)
    dst = torch.empty(bx * rows * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    opts = gic.Options(bc7_quality=args.bc7_quality, bc7_shake_ranks=shake_ranks, bc7_mse_bound=bound)
    gic.encode_device(7, src, size, size, 1, 4, dst, opts, 0, min(rows, 4), stream=stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gic.iter_cap_hits(reset=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    gic.encode_device(7, src, size, size, 1, 4, dst, opts, 0, rows, stream=stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    own = ev0.elapsed_time(ev1)
    t = _max_over_ranks(torch.tensor([wall, own], dtype=torch.float64, device=dev), world)
    wall, kern_ms = float(t[0]), float(t[1])
    spread = _spread_over_ranks(own, world)
    hits = gic.iter_cap_hits(reset=True)
    px = size * rows * 4 * world
    search = "exact (reference search, bit-identical)" if shake_ranks == 0 else \
        f"pruned: {shake_ranks} partitions shaken per mode (per-block MSE tolerance)"
    if bound > 0:
        search = (f"bounded exit: blocks whose mode-6/3/1 probe decodes within MSE {bound:g} are final, the rest " +
                  ("the exact search (contract met by construction)" if shake_ranks == 0 else
                   f"the pruned search ({shake_ranks} partitions; contract checked on a sample)"))
    res = {"metric": f"Mpixels/s BC7 quality {args.bc7_quality:g} (all modes, shakers on), {search}",
           "value": round(px / wall / 1e6, 4), "unit": "Mpixels/s",
           "blocks_per_s": round(bx * rows * world / wall, 1), "ms_per_pass": round(wall * 1e3, 2),
           "kernel_ms": round(kern_ms, 2), "kernel_ms_rank_min_max": [round(x, 2) for x in spread],
           "rows_per_gpu": rows * 4, "dtype": "f64+int32", "iter_cap_hits": hits,
           "roofline": {"bound": "valu", "alg_bytes_per_launch": 80 * bx * rows,
                        "hbm_frac": round(80 * bx * rows / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 8)}}
    if rank == 0 and not args.no_cpu and ref_rows is not None:
        # pruned search: block row 0 against the exact oracle's row (the
        # per-block MSE contract of SURVEY.md 8(d) on the decoded blocks)
        import numpy as np
        import oracle_lib
        got = dst.cpu().numpy().reshape(-1, 16)[:bx]
        host = src.cpu().numpy()[0]
        t = host[0:4, :bx * 4].reshape(4, bx, 4, 4).transpose(1, 0, 2, 3).reshape(bx, 16, 4).astype(np.float64)
        mg = ((oracle_lib.bc7_decode(got).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
        mc = ((oracle_lib.bc7_decode(ref_rows).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
        res["gpu_parity"] = (f"block row 0: {int((got == ref_rows).all(axis=1).sum())}/{bx} bit-identical to the "
                             f"exact oracle, {int((mg > mc * 1.001 + 0.5).sum())} outside the MSE tolerance, "
                             f"mean MSE {mg.mean():.4f} vs {mc.mean():.4f}")
        if bound > 0:
            res["gpu_parity"] += f", {int((mg <= bound).sum())}/{bx} within the exit bound"
    elif rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        threads = _cpu_threads()
        host = src.cpu().numpy()[0]
        c0 = time.perf_counter()
        ref = oracle_lib.encode_image_bc7(host, quality=args.bc7_quality, first_row=0, num_rows=1, threads=threads)
        dt = time.perf_counter() - c0
        got = dst.cpu().numpy().reshape(-1, 16)[:bx]
        same = int((got == ref).all(axis=1).sum())
        res["_ref_row"] = ref
        res["cpu_baseline"] = {"value": round(4 * size / dt / 1e6, 5), "unit": "Mpixels/s", "cores": threads,
                               "kind": "port", "cpu_model": cpu_model(), "sample": f"block row 0 ({bx} blocks, {dt:.1f} s, {threads} threads)",
                               "blocks_per_s": round(bx / dt, 1)}
        res["gpu_parity"] = f"{same}/{bx} blocks of the sampled row bit-identical"
    return res


def _timed(world, dev, stream, fn, steps):
    """Barrier + sync on both sides of `steps` calls of fn; returns
    (max-over-ranks wall s, max-over-ranks event ms per step on `stream`)."""
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    own = ev0.elapsed_time(ev1) / steps
    t = _max_over_ranks(torch.tensor([wall, own], dtype=torch.float64, device=dev), world)
    _timed.spread = _spread_over_ranks(own, world)
    return float(t[0]), float(t[1])


def bc45_leg(args, gic, fmt, world, dev, rank):
    """configs[2]: BC4 on an R8 8192^2 height map (channel 0) or BC5 on its RG8
    normal map; steps x one launch over the rank's whole texture, plus (rank 0)
    a bit-exactness check of 16 block rows against the CPU restatement."""
    import numpy as np
    import torch
    size = args.size
    bx = by = (size + 3) // 4
    src = make_source(fmt, size, rank, dev)
    dst = torch.empty(bx * by * gic.block_bytes(fmt), dtype=torch.uint8, device=dev)
    opts = gic.Options(bc4_channel=0)
    stream = torch.cuda.current_stream(dev)
    ch = CHANNELS[fmt]

    def step():
        gic.encode_device(fmt, src, size, size, 1, ch, dst, opts, 0, by, stream=stream)
    for _ in range(max(1, args.warmup)):
        step()
    wall, kern_ms = _timed(world, dev, stream, step, args.steps)
    alg = ALG_BYTES[fmt] * bx * by
    res = {"metric": f"Mpixels/s {'BC4 R8 height' if fmt == 4 else 'BC5 RG8 normal'} {size}x{size}",
           "value": round(size * size * world * args.steps / wall / 1e6, 3), "unit": "Mpixels/s",
           "ms_per_step": round(wall / args.steps * 1e3, 4), "kernel_ms": round(kern_ms, 4),
           "kernel_ms_rank_min_max": [round(x, 4) for x in _timed.spread],
           "roofline": {"bound": "hbm", "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                        "alg_bytes_per_launch": alg}}
    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        host = src.cpu().numpy()[0]
        rows = 16
        threads = _cpu_threads()
        c0 = time.perf_counter()
        ref = oracle_lib.encode_image(fmt, host, bc4_channel=0, first_row=0, num_rows=rows, threads=threads)
        dt = time.perf_counter() - c0
        budget = args.cpu_seconds / 2   # grow the sample to ~budget s of CPU work, bounded by the image
        if dt < budget / 4 and rows < by:
            rows = int(min(by, max(rows, rows * budget / max(dt, 1e-3))))
            c0 = time.perf_counter()
            ref = oracle_lib.encode_image(fmt, host, bc4_channel=0, first_row=0, num_rows=rows, threads=threads)
            dt = time.perf_counter() - c0
        got = dst.cpu().numpy().reshape(-1, gic.block_bytes(fmt))[:rows * bx]
        res["cpu_baseline"] = {"value": round(rows * 4 * size / dt / 1e6, 4), "unit": "Mpixels/s",
                               "cores": threads, "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"block rows 0-{rows - 1} ({rows * bx} blocks, {dt:.2f} s, {threads} threads)"}
        res["gpu_parity"] = "bit-exact" if np.array_equal(got, ref) else \
            f"{int((got != ref).any(axis=1).sum())} blocks differ"
    return res


def bc7enc16_leg(args, gic, src, size, world, dev, rank, fast):
    """The reference's fast BC7 path (bc7enc16, Image_CompressRichGel999BC7,
    richgel999_bc7enc16.cpp:21-71; ImageCompress_Compress(DXBC7, fast=true)) on
    the same 8K G1 texture: steps x one launch over the rank's whole texture,
    plus (rank 0) a bounded CPU-restatement sample with a bit-exactness check."""
    import numpy as np
    import torch
    bx = by = (size + 3) // 4
    dst = torch.empty(bx * by * 16, dtype=torch.uint8, device=dev)
    opts = gic.Options.bc7enc16(fast=fast, perceptual=True)
    stream = torch.cuda.current_stream(dev)

    def step():
        gic.encode_device(gic.FMT_BC7ENC16, src, size, size, 1, 4, dst, opts, 0, by, stream=stream)
    for _ in range(max(1, args.warmup)):
        step()
    wall, kern_ms = _timed(world, dev, stream, step, args.steps)
    alg = ALG_BYTES[7] * bx * by
    res = {"metric": f"Mpixels/s BC7 by bc7enc16 (the reference's fast BC7 path), perceptual, "
                     f"uber level {0 if fast else 4} ({'fast = true' if fast else 'image-API default'})",
           "value": round(size * size * world * args.steps / wall / 1e6, 3), "unit": "Mpixels/s",
           "blocks_per_s": round(bx * by * world * args.steps / wall, 1),
           "ms_per_step": round(wall / args.steps * 1e3, 4), "kernel_ms": round(kern_ms, 4), "dtype": "f32+int32",
           "kernel_ms_rank_min_max": [round(x, 4) for x in _timed.spread],
           "roofline": {"bound": "valu", "achieved": round(alg / (kern_ms * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
                        "alg_bytes_per_launch": alg}}
    valu = _valu_roofline("valu_bc7enc16_fast.json" if fast else "valu_bc7enc16.json", size, size, kern_ms)
    if valu is not None:
        res["roofline"]["valu"] = valu
    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        host = src.cpu().numpy()[0]
        threads = _cpu_threads()
        rows = 4
        c0 = time.perf_counter()
        ref = oracle_lib.encode_image_bc7enc_rows(host, 0, rows, threads=threads, fast=fast, perceptual=True)
        dt = time.perf_counter() - c0
        budget = args.cpu_seconds / 2   # grow the sample to ~budget s of CPU work, bounded by the image
        if dt < budget / 4:
            rows = int(min(by, max(rows, rows * budget / max(dt, 1e-3))))
            c0 = time.perf_counter()
            ref = oracle_lib.encode_image_bc7enc_rows(host, 0, rows, threads=threads, fast=fast, perceptual=True)
            dt = time.perf_counter() - c0
        got = dst.cpu().numpy().reshape(-1, 16)[:rows * bx]
        res["cpu_baseline"] = {"value": round(rows * 4 * size / dt / 1e6, 4), "unit": "Mpixels/s", "cores": threads,
                               "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"block rows 0-{rows - 1} ({rows * bx} blocks, {dt:.2f} s, {threads} threads)"}
        res["gpu_parity"] = "bit-exact" if np.array_equal(got, ref) else \
            f"{int((got != ref).any(axis=1).sum())} blocks differ"
    return res


def bc6h_leg(args, gic, world, dev, rank, signed=False):
    """BC6H (BC6HBlockEncoder at the image API's quality 1.0;
    unsigned half floats, or signed for a signed source) on a synthetic HDR
    float32 texture (synth.hdr_rgba: 12 stops, noise, highlights; signed: a
    sign from a hash), steps x one launch over the rank's texture, plus (rank
    0) the CPU restatement on a bounded sample of whole blocks with a
    bit-exactness check."""
    import numpy as np
    import torch
    from gfx_imagecompress_amd import synth
    n = args.bc6h_size
    bx = by = (n + 3) // 4
    img = synth.hdr_rgba(n, n, seed=1 + rank, signed=signed)
    src = torch.from_numpy(img.reshape(-1).copy()).to(dev)
    dst = torch.empty(bx * by * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    fmt = gic.FMT_BC6H_SF if signed else gic.FMT_BC6H

    def step():
        gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, n, n, 1, 4, dst, stream=stream)
    step()
    steps = max(1, min(args.steps, 3))
    gic.iter_cap_hits(reset=True)
    wall, kern_ms = _timed(world, dev, stream, step, steps)
    hits = gic.iter_cap_hits(reset=True)
    res = {"metric": f"Mpixels/s BC6H ({'signed' if signed else 'unsigned'}, quality 1.0) on a {n}x{n} synthetic "
                     f"HDR float32 texture",
           "value": round(n * n * world * steps / wall / 1e6, 4), "unit": "Mpixels/s",
           "blocks_per_s": round(bx * by * world * steps / wall, 1), "ms_per_step": round(wall / steps * 1e3, 3),
           "kernel_ms": round(kern_ms, 3), "kernel_ms_rank_min_max": [round(x, 3) for x in _timed.spread],
           "dtype": "f32", "steps": steps, "iter_cap_hits": hits,
           "roofline": {"bound": "valu", "alg_bytes_per_launch": 272 * bx * by,
                        "hbm_frac": round(272 * bx * by / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 8),
                        "note": "272 B per block: 256 B of float32 RGBA texels read, 16 B written"}}
    valu = _valu_roofline("valu_bc6h_shake_signed.json" if signed else "valu_bc6h_shake.json", n, n, kern_ms,
                          launch_key="bc6h_ms")
    if valu is not None:
        res["roofline"]["valu"] = valu
    if rank == 0 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        threads = _cpu_threads()
        # whole blocks of block rows 0-3 (the edge clamp of ReadNxNBlockF for a ragged size)
        rows = min(by, 4)
        ys = np.minimum(np.arange(rows * 4), n - 1)
        xs = np.minimum(np.arange(bx * 4), n - 1)
        t = img[ys][:, xs]
        blocks = t.reshape(rows, 4, bx, 4, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 64)
        nsamp = min(len(blocks), 1024)
        c0 = time.perf_counter()
        ref, _ = oracle_lib.bc6h_blocks(blocks[:nsamp], signed=signed, threads=threads)
        dt = time.perf_counter() - c0
        got = dst.cpu().numpy().reshape(-1, 16)[:nsamp]
        res["cpu_baseline"] = {"value": round(nsamp * 16 / dt / 1e6, 5), "unit": "Mpixels/s", "cores": threads,
                               "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"the first {nsamp} blocks of block rows 0-{rows - 1} ({dt:.2f} s, "
                                         f"{threads} threads)",
                               "blocks_per_s": round(nsamp / dt, 1)}
        res["gpu_parity"] = "bit-exact" if np.array_equal(got, ref) else \
            f"{int((got != ref).any(axis=1).sum())} blocks differ"
    return res


def _valu_roofline(name, size, rows, kern_ms, launch_key=None):
    """VALU issue roofline of a kernel: SQ_INSTS_VALU per launch from the
    committed PMC summary profiles/<name> (tools/valu_json.py, same workload)
    over this run's measured launch duration; None when absent or for another
    workload size."""
    vj = os.path.join(ROOT, "profiles", name)
    try:
        with open(vj) as f:
            vr = json.load(f)
        if vr.get("size") != size or vr.get("rows") != rows:
            return None
        insts = vr["valu_insts_per_launch"] if launch_key is None else vr["valu_insts_per_step"]
        rate = insts / (kern_ms * 1e-3)
        return {"bound": "valu", "achieved": round(rate / 1e12, 4), "peak": round(VALU_PEAK / 1e12, 4),
                "unit": "T wave-instr/s", "frac": round(rate / VALU_PEAK, 4),
                "insts_per_launch": insts, "kernel": vr.get("kernel", "")[:60],
                "source": os.path.relpath(vj, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def _cpu_threads():
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    return max(1, min(threads, os.cpu_count() or 1, 64))


def _batch_check_rows(S, by):
    """(slice, block row) pairs the batch legs check against the oracle: slices
    spread over the stack, the middle row, a shard-chunk boundary row and the
    last row."""
    return sorted({(0, by // 2), (S // 2, max(0, min(by - 1, 16 * (by // 32) - 1))), (S - 1, by - 1)})


def _batch_oracle(args, S, n, bx, by, cache):
    """The exact oracle's blocks of the check rows (computed once per run,
    shared by the exact and the bounded legs) and the CPU time they took."""
    if "rows" in cache:
        return cache["rows"], cache["dt"], cache["threads"]
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    from gfx_imagecompress_amd import synth
    threads = _cpu_threads()
    rows, dt = {}, 0.0
    for sl, row in _batch_check_rows(S, by):
        img = synth.g1(n, n, seed=0x9E3779B9 + sl)
        c0 = time.perf_counter()
        rows[(sl, row)] = (oracle_lib.encode_image_bc7(img, quality=args.bc7_quality, first_row=row, num_rows=1,
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
        src = synth.g1_torch(n, n, S, seed=0x9E3779B9, device=dev)
    dst = torch.empty(max(1, nblk * 16), dtype=torch.uint8, device=dev)
    opts = gic.Options(bc7_quality=args.bc7_quality, bc7_shake_ranks=shake_ranks, bc7_mse_bound=bound)
    stream = torch.cuda.current_stream(dev)
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
        search = (f"bounded exit: blocks whose mode-6/3/1 probe decodes within MSE {bound:g} are final, the rest "
                  f"{'the exact search (contract met by construction)' if shake_ranks == 0 else 'the pruned search'}")
    else:
        search = ("exact (the reference search)" if shake_ranks == 0 else
                  f"pruned, {shake_ranks} partitions shaken per mode (per-block MSE tolerance)")
    res = {
        "metric": f"Mpixels/s BC7 quality {args.bc7_quality:g} on the configs[4] batch, {search}",
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
        "roofline": {"bound": "valu", "achieved": round(80 * nblk / (kern_ms * 1e-3) / 1e9, 4),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(80 * nblk / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 8),
                     "traffic": None, "alg_bytes_per_launch": 80 * nblk,
                     "note": "VALU bound; HBM fraction (80 B per block) per BASELINE.json"},
        "cpu_baseline": None,
    }
    host = full.cpu().numpy().reshape(S, by, bx, 16) if full is not None and \
        full.numel() >= total_blocks * 16 else None
    if not args.no_cpu and host is not None:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        rows, dt, threads = _batch_oracle(args, S, n, bx, by, oracle_cache if oracle_cache is not None else {})
        same = bad = tot = 0
        mse_g = mse_c = 0.0
        for (sl, row), (ref, texels) in rows.items():
            got = host[sl, row]
            same += int((got == ref).all(axis=1).sum())
            tot += bx
            t = texels.reshape(4, bx, 4, 4).transpose(1, 0, 2, 3).reshape(bx, 16, 4).astype(np.float64)
            mg = ((oracle_lib.bc7_decode(got).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
            mc = ((oracle_lib.bc7_decode(ref).astype(np.float64) - t) ** 2).mean(axis=(1, 2))
            bad += int((mg > mc * 1.001 + 0.5).sum())
            mse_g += float(mg.sum())
            mse_c += float(mc.sum())
        where = ", ".join(f"slice {sl} row {row}" for sl, row in rows)
        res["cpu_baseline"] = {"value": round(len(rows) * 4 * n / dt / 1e6, 6), "unit": "Mpixels/s",
                               "cores": threads, "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"the exact search on {len(rows)} block rows ({where}; {tot} blocks, "
                                         f"{dt:.1f} s, {threads} threads)",
                               "blocks_per_s": round(tot / dt, 1)}
        res["gpu_parity"] = (f"{same}/{tot} blocks of {where}{' (after the gather)' if world > 1 else ''} "
                             f"bit-identical to the exact oracle, "
                             f"{bad} outside the per-block MSE contract, mean MSE {mse_g / tot:.4f} vs "
                             f"{mse_c / tot:.4f}")
        if shake_ranks == 0 and bound == 0:
            res["gpu_parity_ok"] = same == tot
        else:
            res["gpu_parity_ok"] = bad == 0
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
    rows = by if not args.rows else min(args.rows, by)
    src = make_source(fmt, size, rank, dev)
    ch = CHANNELS[fmt]
    nblocks = bx * rows
    dst = torch.empty(nblocks * gic.block_bytes(fmt), dtype=torch.uint8, device=dev)
    opts = gic.Options(bc4_channel=0, bc7_quality=args.bc7_quality,
                       bc7_shake_ranks=args.bc7_shake_ranks if fmt == 7 else 0)
    stream = torch.cuda.current_stream(dev)

    def step():
        gic.encode_device(fmt, src, size, size, 1, ch, dst, opts, 0, rows, stream=stream)

    for _ in range(args.warmup):
        step()
    wall, kern_ms = _timed(world, dev, stream, step, args.steps)
    spread = _timed.spread

    gather_ms = None
    if args.gather and world > 1:
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        out_all = _gather_root(dst, world)
        torch.cuda.synchronize(dev)
        gather_ms = (time.perf_counter() - g0) * 1e3
        if out_all is not None and out_all.numel() != world * dst.numel():
            raise RuntimeError("gather returned a wrong size")

    pixels = size * rows * 4 * world          # pixels encoded per step, all ranks
    value = pixels * args.steps / wall / 1e6
    alg_bytes = ALG_BYTES[fmt] * nblocks      # per launch, per rank
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    tj = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_{args.format}.json")
    if os.path.exists(tj):
        try:
            with open(tj) as f:
                tr = json.load(f)
            if tr.get("size") == size and tr.get("rows") == rows * 4:
                traffic = tr.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # VALU issue roofline of the same kernel: SQ_INSTS_VALU per launch from the
    # committed PMC summary (tools/pmc_valu.sh + tools/valu_json.py, same
    # workload) over this run's measured launch duration
    valu = _valu_roofline(f"valu_{args.format}.json", size, rows * 4, kern_ms)

    bc7 = bc7_pruned = None
    bounded = {}
    if fmt == 1 and args.bc7_rows != 0:
        bc7 = bc7_secondary(args, gic, src, size, rows, world, dev, rank)
        ref_row = bc7.pop("_ref_row", None)
        if args.bc7_shake_ranks > 0:
            bc7_pruned = bc7_secondary(args, gic, src, size, rows, world, dev, rank, args.bc7_shake_ranks, ref_row)
        if args.bc7_mse_bound > 0:
            bounded["bc7_bounded"] = bc7_secondary(args, gic, src, size, rows, world, dev, rank, 0, ref_row,
                                                   args.bc7_mse_bound)
            if args.bc7_shake_ranks > 0:
                bounded["bc7_bounded_pruned"] = bc7_secondary(args, gic, src, size, rows, world, dev, rank,
                                                              args.bc7_shake_ranks, ref_row, args.bc7_mse_bound)
    enc16 = {}
    if fmt == 1 and not args.no_bc7enc:
        enc16["bc7enc16"] = bc7enc16_leg(args, gic, src, size, world, dev, rank, fast=False)
        enc16["bc7enc16_fast"] = bc7enc16_leg(args, gic, src, size, world, dev, rank, fast=True)
    bc45 = {}
    if fmt == 1 and not args.no_bc45:
        for f in (4, 5):
            bc45[f"bc{f}"] = bc45_leg(args, gic, f, world, dev, rank)
    if fmt == 1 and args.bc6h_size > 0:
        bc45["bc6h"] = bc6h_leg(args, gic, world, dev, rank)
        bc45["bc6h_signed"] = bc6h_leg(args, gic, world, dev, rank, signed=True)
    batch = {}
    if fmt == 1 and not args.no_batch:
        # configs[4] at its size: the 64 x 4096^2 G1 stack, one pass each of the
        # bounded exit (exact survivors) and the exact reference search, block
        # rows dealt over the ranks, one gather to rank 0, oracle rows checked
        from gfx_imagecompress_amd import synth
        bsrc = synth.g1_torch(args.batch_size, args.batch_size, args.batch_slices, seed=0x9E3779B9, device=dev)
        cache = {}
        batch["batch64_bounded"] = batch_run(args, gic, world, rank, dev, args.bc7_mse_bound or 0.5, 0, 1, 0,
                                             src=bsrc, oracle_cache=cache)
        if not args.no_batch_exact:
            batch["batch64_exact"] = batch_run(args, gic, world, rank, dev, 0.0, 0, 1, 0, src=bsrc,
                                               oracle_cache=cache)
        del bsrc
        torch.cuda.empty_cache()

    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu:
        host = src.cpu().numpy()[0]
        torch.cuda.synchronize(dev)
        cpu, parity, mism = cpu_baseline(fmt, host, size, dst.cpu().numpy(), args.cpu_seconds, rows, args.bc7_quality)
        cpu["gpu_parity"] = "bit-exact" if parity else f"{mism} blocks differ"
        cpu["cpu_model"] = cpu_model()

    if rank == 0:
        line = {
            "metric": "Mpixels/s (and blocks/s) BC1 & BC7 on 8K RGBA8 at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if fmt != 7 else "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.format.upper()} default quality, {size}x{size * world} synthetic "
                                   f"{'RGBA8 G1 gradient+noise' if fmt in (1, 7) else ('R8 height' if fmt == 4 else 'RG8 normal')}"
                                   f", block-row shards of {size}x{rows * 4} per GPU",
                       "format": args.format.upper(), "width": size, "rows_per_gpu": rows * 4,
                       "global_batch_blocks": nblocks * world, "parallelism": f"block-row shards x{world}",
                       "world_size_seen": dist.get_world_size() if world > 1 else 1},
            "blocks_per_s": round(nblocks * world * args.steps / wall, 1),
            "kernel_ms": round(kern_ms, 4),
            "kernel_ms_rank_min_max": [round(x, 4) for x in spread],
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes,
                         "note": "compute (VALU) bound; HBM fraction reported per BASELINE.json, the "
                                 "binding VALU issue fraction in roofline.valu"},
            "cpu_baseline": cpu,
        }
        if valu is not None:
            line["roofline"]["valu"] = valu
        if gather_ms is not None:
            line["gather_ms"] = round(gather_ms, 3)
        if bc7 is not None:
            line["bc7"] = bc7
        if bc7_pruned is not None:
            line["bc7_pruned"] = bc7_pruned
        line.update(bounded)
        line.update(enc16)
        line.update(bc45)
        line.update(batch)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
