"""Block-row sharding of one image stack across ranks.

Every 4x4 block is independent (a fresh encoder per block,
amd_bc7_compressor.cpp:19), so rank r of N encodes the contiguous block rows
``shard_rows(BY, N, r)`` of every slice into its own buffer with
``gic_hip_encode_rows`` -- no collective in the data path.  When one process
needs the whole bitstream, ``gather_blocks`` collects the shards with a single
all-gather (RCCL over xGMI on GPUs, gloo in the CPU tests) and
``assemble`` restores the reference's row-major-per-slice block order
(Image_GetBlockIndex, block_utils.cpp:157-159).
"""
from __future__ import annotations


def shard_rows(block_rows: int, world: int, rank: int) -> tuple[int, int]:
    """(first block row, number of block rows) of ``rank``; the first
    ``block_rows % world`` ranks take one extra row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(block_rows, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def encode_shard(fmt: int, src, width: int, height: int, slices: int, channels: int, rank: int, world: int,
                 options=None, stream=None, encoder=None):
    """Encode this rank's block rows of every slice.

    Returns a uint8 tensor of ``slices * rows * bx`` blocks on ``src``'s device.
    ``encoder`` defaults to the HIP path (``gfx_imagecompress_amd.encode_device``);
    tests substitute a CPU checker with the same signature.
    """
    import torch
    from . import blocks_shape, block_bytes, encode_device
    bx, by = blocks_shape(width, height)
    first, rows = shard_rows(by, world, rank)
    dst = torch.empty(max(1, bx * rows * slices * block_bytes(fmt)), dtype=torch.uint8, device=src.device)
    if rows:
        (encoder or encode_device)(fmt, src, width, height, slices, channels, dst, options,
                                   first_block_row=first, num_block_rows=rows, stream=stream)
    return dst[: bx * rows * slices * block_bytes(fmt)]


def gather_blocks(local, fmt: int, width: int, height: int, slices: int, world: int, group=None):
    """All-gather every rank's shard (padded to the largest shard) and return
    the whole stack's blocks in reference order."""
    import torch
    import torch.distributed as dist
    from . import blocks_shape, block_bytes
    bx, by = blocks_shape(width, height)
    bb = block_bytes(fmt)
    most = shard_rows(by, world, 0)[1] * bx * slices * bb
    pad = torch.zeros(max(most, 1), dtype=torch.uint8, device=local.device)
    pad[: local.numel()] = local
    out = torch.empty(world * pad.numel(), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = [out[r * pad.numel(): r * pad.numel() + shard_rows(by, world, r)[1] * bx * slices * bb]
             for r in range(world)]
    return assemble(parts, fmt, width, height, slices)


def assemble(parts, fmt: int, width: int, height: int, slices: int):
    """Interleave per-rank shards ([slices][rows_r][bx] blocks each) into
    [slices][BY][bx] order."""
    import torch
    from . import blocks_shape, block_bytes
    bx, by = blocks_shape(width, height)
    bb = block_bytes(fmt)
    world = len(parts)
    views = []
    for r, p in enumerate(parts):
        rows = shard_rows(by, world, r)[1]
        views.append(p.reshape(slices, rows * bx * bb))
    return torch.cat(views, dim=1).reshape(-1)
