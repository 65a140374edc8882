"""configs[4] at its workload: full 4096^2 G1 slices (slice s seeded
0x9E3779B9 + s), BC7, encoded as 8 simulated rank shards through
gic_hip_encode_rows and reassembled with shard.assemble -- the multi-GPU data
path of SURVEY.md 8(e) on one device (one call per rank range, every slice at
once, as each rank of bench.py --workload batch64 does).

* The reassembly is byte-identical to a single-call encode of the stack
  (contiguous shards and round-robin chunks of 16 block rows).
* Every block decodes (GPU decoder); the exact search emits modes <= 5 on the
  opaque G1 slices (colourRestrict, amd_bc7_body.cpp:1340-1380) at PSNR > 40.
* Block rows on both sides of the shard boundaries (127/128, 895/896 with
  8 ranks of 128 rows) of several slices equal the oracle bit-for-bit (exact
  search) or meet the per-block MSE contract MSE <= MSE_ref * (1 + 1e-3) + 0.5
  (bounded exit), on 16-block crops (interior crops: the oracle's blocks are
  the same as on the whole slice).

Reference: the slice loop of Image_CompressAMDBC7, amd_bc7_compressor.cpp:44-77.
"""
import numpy as np
import pytest

import gfx_imagecompress_amd as gic
import oracle_lib
from gfx_imagecompress_amd import shard, synth

pytestmark = pytest.mark.gpu

N = 4096
BX = BY = N // 4
WORLD = 8
SEED = 0x9E3779B9
BOUNDARY_ROWS = (127, 128, 895, 896)
MSE_REL, MSE_ABS = 1e-3, 0.5


def _encode_stack(src, slices, opts):
    import torch
    dst = torch.empty(slices * BX * BY * 16, dtype=torch.uint8, device=src.device)
    gic.encode_device(gic.FMT_BC7, src, N, N, slices, 4, dst, opts)
    return dst


def _encode_sharded(src, slices, opts, chunk):
    parts = [shard.encode_shard(gic.FMT_BC7, src, N, N, slices, 4, r, WORLD, opts, chunk=chunk)
             for r in range(WORLD)]
    for r, p in enumerate(parts):
        assert p.numel() == shard.shard_blocks(BY, BX, slices, WORLD, r, chunk) * 16
    return shard.assemble(parts, gic.FMT_BC7, N, N, slices, chunk)


def _decode_psnr(blocks, src, slices):
    """GPU decode of the whole stack; per-block MSE (RGBA, 0..255) and per-slice PSNR."""
    import torch
    out = torch.empty(slices * N * N * 4, dtype=torch.uint8, device=src.device)
    gic.decode_device(gic.FMT_BC7, blocks, N, N, slices, out)
    d = out.view(slices, BY, 4, BX, 4, 4).to(torch.float32) - src.view(slices, BY, 4, BX, 4, 4).to(torch.float32)
    blk = (d * d).sum(dim=(2, 4, 5)) / 64.0              # (slices, BY, BX)
    mse = blk.mean(dim=(1, 2)).double()
    psnr = 10.0 * torch.log10(255.0 ** 2 / mse)
    return blk, psnr.cpu().numpy()


def _modes(blocks):
    b0 = blocks.view(-1, 16)[:, 0].cpu().numpy().astype(np.int64)
    mode = np.full(b0.shape, 8, np.int64)                 # 8 = reserved (no bit set)
    for m in range(7, -1, -1):
        mode[(b0 >> m) & 1 == 1] = m
    return mode


def _crop_cols(sl):
    """A 16-block column range per slice, spread over the width."""
    c0 = (sl * 97) % (BX - 16)
    return c0, c0 + 16


def _oracle_rows(slices):
    """Exact-search oracle of the boundary rows of each slice on its 16-block
    crop, all crops as the slices of one stack (the oracle's thread pool works
    per (slice, block row)).  Returns {(slice, row): (blocks, crop texels)}."""
    crops, keys = [], []
    for sl in slices:
        img = synth.g1(N, N, seed=SEED + sl)
        c0, c1 = _crop_cols(sl)
        for row in BOUNDARY_ROWS:
            crops.append(img[4 * row:4 * row + 4, 4 * c0:4 * c1])
            keys.append((sl, row))
    stack = np.ascontiguousarray(np.stack(crops))
    ref = oracle_lib.encode_image_bc7(stack).reshape(len(keys), 16, 16)
    return {k: (ref[i], stack[i]) for i, k in enumerate(keys)}


def _crop_mse(blocks, crop):
    t = crop.reshape(4, -1, 4, 4).transpose(1, 0, 2, 3).reshape(-1, 16, 4).astype(np.float64)
    return ((oracle_lib.bc7_decode(blocks).astype(np.float64) - t) ** 2).mean(axis=(1, 2))


def test_bc7_batch_shards_exact(gpu):
    """4 full 4096^2 slices, the exact (reference) search: 8 contiguous rank
    shards reassemble to the single-call encode; boundary rows bit-identical to
    the oracle."""
    import torch
    S = 4
    src = synth.g1_torch(N, N, S, seed=SEED, device=gpu)
    opts = gic.Options()
    whole = _encode_stack(src, S, opts)
    sharded = _encode_sharded(src, S, opts, chunk=0)
    torch.cuda.synchronize()
    assert torch.equal(whole, sharded), \
        f"{int((whole.view(-1, 16) != sharded.view(-1, 16)).any(dim=1).sum())} blocks differ after reassembly"
    modes = _modes(whole)
    assert modes.max() <= 5, f"modes {np.unique(modes).tolist()} on opaque slices"
    _, psnr = _decode_psnr(whole, src, S)
    assert (psnr > 40).all(), psnr.tolist()
    host = whole.view(S, BY, BX, 16).cpu().numpy()
    for (sl, row), (ref, _) in _oracle_rows((0, S - 1)).items():
        cols = _crop_cols(sl)
        got = host[sl, row, cols[0]:cols[1]]
        bad = np.nonzero((got != ref).any(axis=1))[0]
        assert len(bad) == 0, f"slice {sl} row {row}: blocks {(bad + cols[0]).tolist()} differ from the oracle"


def test_bc7_batch64_bounded_shards(gpu):
    """The whole 64 x 4096^2 stack under the bounded exit (bc7_mse_bound 0.5,
    exact survivors): 8 rank shards in round-robin chunks of 16 block rows
    reassemble to the single-call encode; every block decodes within the bound
    or is a full-search block; boundary rows meet the MSE contract against the
    exact oracle."""
    import torch
    S = 64
    src = synth.g1_torch(N, N, S, seed=SEED, device=gpu)
    opts = gic.Options(bc7_mse_bound=0.5)
    whole = _encode_stack(src, S, opts)
    sharded = _encode_sharded(src, S, opts, chunk=16)
    torch.cuda.synchronize()
    assert torch.equal(whole, sharded), \
        f"{int((whole.view(-1, 16) != sharded.view(-1, 16)).any(dim=1).sum())} blocks differ after reassembly"
    del sharded
    modes = _modes(whole)
    assert modes.max() <= 7
    blk, psnr = _decode_psnr(whole, src, S)
    assert (psnr > 40).all(), psnr.tolist()
    within = float((blk <= 0.5).double().mean())
    assert within > 0.9, f"only {within:.3f} of the blocks decode within the exit bound"
    host = whole.view(S, BY, BX, 16).cpu().numpy()
    del whole, blk
    for (sl, row), (ref, crop) in _oracle_rows((0, 31, S - 1)).items():
        cols = _crop_cols(sl)
        got = host[sl, row, cols[0]:cols[1]]
        mg, mc = _crop_mse(got, crop), _crop_mse(ref, crop)
        bad = np.nonzero(mg > mc * (1 + MSE_REL) + MSE_ABS)[0]
        assert len(bad) == 0, f"slice {sl} row {row}: blocks {(bad + cols[0]).tolist()} outside the contract"
        # a block outside the bound is the exact search's own block
        off = np.nonzero(mg > 0.5)[0]
        assert (got[off] == ref[off]).all(), f"slice {sl} row {row}: a full-search block differs"
