"""Block-row sharding of one image stack across ranks.

Every 4x4 block is independent (a fresh encoder per block,
amd_bc7_compressor.cpp:19), so rank r of N encodes its block rows of every
slice into its own buffer with ``gic_hip_encode_rows`` -- no collective in the
data path.  Two row assignments:

* contiguous (``chunk = 0``, the default): rank r takes ``shard_rows(BY, N, r)``,
  one range per rank;
* interleaved (``chunk = C > 0``): the block rows are cut into chunks of C rows
  dealt round-robin, rank r taking chunks r, r + N, r + 2N, ... -- the cyclic
  chunking SURVEY.md 8(e) / 7 H5 suggests when content makes some rows much
  costlier than others (the BC7 bounded exit: a noisy region's blocks run the
  full search at ~100x the cost of a probe-final block).

A rank's buffer holds its ranges one after another, each range as
[slices][rows][bx] blocks (one ``gic_hip_encode_rows`` call per range).  When
one process needs the whole bitstream, ``gather_to_root`` collects the shards
with a single gather to rank 0 (RCCL over xGMI on GPUs, gloo in the CPU tests)
and ``assemble`` restores the reference's row-major-per-slice block order
(Image_GetBlockIndex, block_utils.cpp:157-159).
"""
from __future__ import annotations


def shard_rows(block_rows: int, world: int, rank: int) -> tuple[int, int]:
    """(first block row, number of block rows) of ``rank`` in the contiguous
    split; the first ``block_rows % world`` ranks take one extra row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(block_rows, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def row_ranges(block_rows: int, world: int, rank: int, chunk: int = 0) -> list[tuple[int, int]]:
    """The (first, rows) ranges of ``rank``, in buffer order: one contiguous
    range (chunk 0) or the chunks r, r + N, ... of ``chunk`` rows (the last
    chunk of the image may be short; adjacent chunks, as with one rank, merge
    into one range).  Empty ranges are omitted."""
    if chunk < 0:
        raise ValueError(f"bad chunk {chunk}")
    if not chunk:
        first, rows = shard_rows(block_rows, world, rank)
        return [(first, rows)] if rows else []
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    out = []
    for first in range(rank * chunk, block_rows, world * chunk):
        n = min(chunk, block_rows - first)
        if out and out[-1][0] + out[-1][1] == first:   # adjacent chunks (one rank) form one range
            out[-1] = (out[-1][0], out[-1][1] + n)
        else:
            out.append((first, n))
    return out


def shard_blocks(block_rows: int, bx: int, slices: int, world: int, rank: int, chunk: int = 0) -> int:
    """Blocks in ``rank``'s buffer."""
    return sum(n for _, n in row_ranges(block_rows, world, rank, chunk)) * bx * slices


def encode_shard(fmt: int, src, width: int, height: int, slices: int, channels: int, rank: int, world: int,
                 options=None, stream=None, encoder=None, chunk: int = 0, dst=None):
    """Encode this rank's block rows of every slice (one encoder call per range).

    Returns a uint8 tensor of ``shard_blocks(...)`` blocks on ``src``'s device
    (a view of ``dst`` when given).  ``encoder`` defaults to the HIP path
    (``gfx_imagecompress_amd.encode_device``); tests substitute a CPU checker
    with the same signature.
    """
    import torch
    from . import blocks_shape, block_bytes, encode_device
    bx, by = blocks_shape(width, height)
    bb = block_bytes(fmt)
    total = shard_blocks(by, bx, slices, world, rank, chunk) * bb
    if dst is None:
        dst = torch.empty(max(1, total), dtype=torch.uint8, device=src.device)
    elif dst.numel() < total:
        raise ValueError(f"dst holds {dst.numel()} bytes, the shard needs {total}")
    off = 0
    for first, rows in row_ranges(by, world, rank, chunk):
        n = rows * bx * slices * bb
        (encoder or encode_device)(fmt, src, width, height, slices, channels, dst[off:off + n], options,
                                   first_block_row=first, num_block_rows=rows, stream=stream)
        off += n
    return dst[:total]


def gather_to_root(local, fmt: int, width: int, height: int, slices: int, world: int, chunk: int = 0,
                   root: int = 0, group=None):
    """One gather of every rank's shard (padded to the largest) to ``root``:
    ``torch.distributed.gather`` -- RCCL's grouped send/recv on device tensors,
    gloo on host tensors.  Returns the whole stack's blocks in reference order
    on ``root`` and None elsewhere."""
    import torch
    import torch.distributed as dist
    from . import blocks_shape, block_bytes
    bx, by = blocks_shape(width, height)
    bb = block_bytes(fmt)
    sizes = [shard_blocks(by, bx, slices, world, r, chunk) * bb for r in range(world)]
    most = max(1, max(sizes))
    gloo = dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if gloo else local.device
    pad = torch.zeros(most, dtype=torch.uint8, device=dev)
    pad[: local.numel()] = local.to(dev)
    rank = dist.get_rank(group)
    bufs = [torch.empty(most, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == root else None
    dist.gather(pad, gather_list=bufs, dst=root, group=group)
    if rank != root:
        return None
    return assemble([b[:n] for b, n in zip(bufs, sizes)], fmt, width, height, slices, chunk)


def gather_blocks(local, fmt: int, width: int, height: int, slices: int, world: int, group=None, chunk: int = 0):
    """All-gather variant (every rank receives the whole stack): for callers
    where each process needs the full bitstream.  The bench and the
    multi-GPU path use ``gather_to_root``."""
    import torch
    import torch.distributed as dist
    from . import blocks_shape, block_bytes
    bx, by = blocks_shape(width, height)
    bb = block_bytes(fmt)
    sizes = [shard_blocks(by, bx, slices, world, r, chunk) * bb for r in range(world)]
    most = max(1, max(sizes))
    pad = torch.zeros(most, dtype=torch.uint8, device=local.device)
    pad[: local.numel()] = local
    out = torch.empty(world * most, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = [out[r * most: r * most + sizes[r]] for r in range(world)]
    return assemble(parts, fmt, width, height, slices, chunk)


def assemble(parts, fmt: int, width: int, height: int, slices: int, chunk: int = 0):
    """Place per-rank shards (each its ranges in order, a range as
    [slices][rows][bx] blocks) into [slices][BY][bx] order."""
    import torch
    from . import blocks_shape, block_bytes
    bx, by = blocks_shape(width, height)
    bb = block_bytes(fmt)
    world = len(parts)
    if not parts:
        raise ValueError("no shards")
    out = torch.empty((slices, by, bx * bb), dtype=torch.uint8, device=parts[0].device)
    for r, p in enumerate(parts):
        off = 0
        for first, rows in row_ranges(by, world, r, chunk):
            n = slices * rows * bx * bb
            if p.numel() < off + n:
                raise ValueError(f"shard {r} holds {p.numel()} bytes, expected at least {off + n}")
            out[:, first:first + rows] = p[off:off + n].reshape(slices, rows, bx * bb)
            off += n
    return out.reshape(-1)
