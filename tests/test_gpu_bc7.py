"""GPU parity tests for BC7 (configs 4-5) against the oracle.

Contract: per-block MSE_gpu <= MSE_cpu * (1 + 1e-3) + 0.5 on
the decoded RGBA (0..255), with the share of bit-identical blocks reported.
The kernels are written to be bit-exact, so the tests also assert identity
where the oracle is the same arithmetic.
"""
import os

import numpy as np
import pytest

import gfx_imagecompress_amd as gic
import oracle_lib
from gfx_imagecompress_amd import synth
from test_gpu_parity import GOLDEN, _golden_case, _manifest, gpu_encode, _mismatch_report

pytestmark = pytest.mark.gpu

MSE_REL, MSE_ABS = 1e-3, 0.5   # per-block tolerance written into the contract


def _block_mse(blocks, src_blocks):
    dec = oracle_lib.bc7_decode(blocks).astype(np.float64)
    return ((dec - src_blocks.astype(np.float64)) ** 2).mean(axis=(1, 2))


def _src_blocks(img, first_row=0, num_rows=None):
    a = img if img.ndim == 3 else img[..., None]
    h, w, c = a.shape
    if c < 4:
        pad = np.zeros((h, w, 4), np.uint8)
        pad[..., :c] = a
        pad[..., 3] = 255
        a = pad
    bx, by = (w + 3) // 4, (h + 3) // 4
    rows = by - first_row if num_rows is None else num_rows
    ys = np.minimum(np.arange(first_row * 4, (first_row + rows) * 4), h - 1)
    xs = np.minimum(np.arange(bx * 4), w - 1)
    t = a[ys][:, xs]
    return t.reshape(rows, 4, bx, 4, 4).transpose(0, 2, 1, 3, 4).reshape(rows * bx, 16, 4)


def check_tolerance(gpu_blocks, cpu_blocks, src_blocks):
    mg = _block_mse(gpu_blocks, src_blocks)
    mc = _block_mse(cpu_blocks, src_blocks)
    bad = np.nonzero(mg > mc * (1 + MSE_REL) + MSE_ABS)[0]
    assert len(bad) == 0, f"{len(bad)} blocks exceed the MSE tolerance, first {bad[:8].tolist()}"
    return float((gpu_blocks == cpu_blocks).all(axis=1).mean())


@pytest.mark.parametrize("name", sorted(k for k in _manifest() if k.startswith("bc7")))
def test_golden_bc7(gpu, name):
    fmt, img, kw = _golden_case(name)
    out = gpu_encode(fmt, img, None, first_row=kw.get("first_row", 0), num_rows=kw.get("num_rows"))
    ref = np.fromfile(os.path.join(GOLDEN, name + ".bin"), np.uint8).reshape(out.shape)
    check_tolerance(out, ref, _src_blocks(img, kw.get("first_row", 0), kw.get("num_rows")))
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


def test_bc7_block_errors_match_oracle(gpu):
    img = synth.g1(64, 16)
    out, err = gpu_encode(7, img, err=True)
    ref, rerr = oracle_lib.encode_image(7, img, want_err=True)
    assert np.array_equal(out, ref), _mismatch_report(out, ref)
    assert np.array_equal(err, rerr)


def _gpu_blocks_f32(blocks, mode_mask=0xFF):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(blocks, np.float32).reshape(-1, 64)).cuda()
    dst = torch.zeros(t.shape[0] * 16, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_f32(gic.FMT_BC7, t, dst, gic.Options(bc7_mode_mask=mode_mask))
    torch.cuda.synchronize()
    return dst.cpu().numpy().reshape(-1, 16)


@pytest.mark.parametrize("mask", [0xFF, 0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x00, 0xC0])
def test_bc7_mode_masks(gpu, mask):
    rng = np.random.default_rng(mask + 1)
    blocks = []
    for k in range(12):
        b = rng.integers(0, 256, (16, 4)).astype(np.float32)
        if k % 3 == 0:
            b[:, 3] = 255
        if k % 4 == 1:
            b[:] = b[0]            # solid
        blocks.append(b / np.float32(255.0))
    blocks = np.stack(blocks)
    got = _gpu_blocks_f32(blocks, mask)
    for i, b in enumerate(blocks):
        enc, _ = oracle_lib.bc7_block(b, mask)
        assert got[i].tobytes() == enc, (mask, i)


def test_bc7_arbitrary_float_blocks(gpu):
    """Non-integer inputs exercise the f64 shaker path."""
    rng = np.random.default_rng(17)
    blocks = rng.random((16, 16, 4), dtype=np.float32)
    blocks[::2, :, 3] = 1.0
    got = _gpu_blocks_f32(blocks)
    for i, b in enumerate(blocks):
        enc, _ = oracle_lib.bc7_block(b)
        assert got[i].tobytes() == enc, i


def test_bc7_reference_patterns(gpu):
    for img in (synth.reference_pattern_rgb(32, 32), synth.reference_pattern_rgb(32, 32, punch_through=True),
                synth.reference_pattern_rgb(32, 32, alpha_ramp=True), synth.noise_rgba(13, 11, seed=4, alpha=True)):
        out = gpu_encode(7, img)
        ref = oracle_lib.encode_image(7, img)
        assert np.array_equal(out, ref), _mismatch_report(out, ref)


def test_bc7_8k_sampled_rows(gpu):
    """Config 4 (8192^2 G1, default quality): sampled block rows vs the oracle."""
    n = 8192
    img = synth.g1(n, n)
    for row in (0, 1000, 2047):
        out = gpu_encode(7, img, first_row=row, num_rows=1)[:256]
        ref = oracle_lib.encode_image(7, img, first_row=row, num_rows=1)[:256]
        check_tolerance(out, ref, _src_blocks(img, row, 1)[:256])
        assert np.array_equal(out, ref), _mismatch_report(out, ref)


def test_bc7_4096_seeded_random_blocks(gpu):
    """SURVEY.md 8(d) random-block sample: 4096 seeded blocks of uniform RGBA
    noise (half of them opaque), every block against the oracle."""
    rng = np.random.default_rng(20261015)
    img = rng.integers(0, 256, (256, 256, 4), dtype=np.uint8)
    img[:128, :, 3] = 255
    out = gpu_encode(7, img)
    ref = oracle_lib.encode_image(7, img)
    check_tolerance(out, ref, _src_blocks(img))
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


@pytest.mark.parametrize("quality", [0.0, 0.05, 0.2, 0.45, 0.55, 0.65, 0.75, 0.9])
def test_bc7_quality_levels(gpu, quality):
    """BC7BlockEncoder quality < 1 (block API Image_CompressAMDMultiModeLDRBlock):
    fewer partitions, smaller shake windows, corner search by range, error-
    threshold early exits over partition ranks and modes, quantiser-error
    gating of dual-index candidates (amd_bc7_body.hpp:94-149)."""
    g1 = synth.g1(64, 16)
    noise = synth.noise_rgba(32, 16, seed=7, alpha=True)
    for img in (g1, noise):
        import torch
        src = torch.from_numpy(np.ascontiguousarray(img)[None]).cuda()
        h, w = img.shape[:2]
        nb = ((w + 3) // 4) * ((h + 3) // 4)
        dst = torch.zeros(nb * 16, dtype=torch.uint8, device="cuda")
        gic.encode_device(7, src, w, h, 1, 4, dst, gic.Options(bc7_quality=quality))
        torch.cuda.synchronize()
        out = dst.cpu().numpy().reshape(-1, 16)
        ref = oracle_lib.encode_image_bc7(img, quality=quality)
        assert np.array_equal(out, ref), (quality, _mismatch_report(out, ref))


@pytest.mark.parametrize("performance,quality", [(0.0, 1.0), (0.1, 1.0), (0.5, 1.0), (0.95, 1.0), (0.0, 0.6),
                                                 (0.05, 0.3)])
def test_bc7_performance_levels(gpu, performance, quality):
    """BC7BlockEncoder performance < 1: blocks whose range exceeds 255 *
    performance quantise with the exhaustive optQuantTrace_d (trace tables of
    traceBuilder) instead of optQuantAnD_d -- single-index modes with at most 8
    clusters and both halves of modes 4/5 (amd_bc7_body.cpp:606-633,
    :1103-1154) -- bit-identical to the oracle's restatement."""
    import torch
    g1 = synth.g1(64, 16)
    noise = synth.noise_rgba(32, 16, seed=9, alpha=True)
    for img in (g1, noise):
        src = torch.from_numpy(np.ascontiguousarray(img)[None]).cuda()
        h, w = img.shape[:2]
        nb = ((w + 3) // 4) * ((h + 3) // 4)
        dst = torch.zeros(nb * 16, dtype=torch.uint8, device="cuda")
        gic.encode_device(7, src, w, h, 1, 4, dst, gic.Options(bc7_quality=quality, bc7_performance=performance))
        torch.cuda.synchronize()
        out = dst.cpu().numpy().reshape(-1, 16)
        ref = oracle_lib.encode_image_bc7(img, quality=quality, performance=performance)
        assert np.array_equal(out, ref), (performance, _mismatch_report(out, ref))


def test_bc7_8k_whole_image_properties(gpu):
    """Config 4 at full size (8192^2 G1): every block decodes, only modes 0-5
    appear (opaque non-solid blocks drop 6/7, Q4), the decoded image is close
    to the source, the per-block encoder errors are finite, and a sampled block
    row is bit-identical to the oracle."""
    import torch
    n = 8192
    src = synth.g1_torch(n, n, 1, seed=0x9E3779B9, device="cuda")
    nb = (n // 4) * (n // 4)
    dst = torch.empty(nb * 16, dtype=torch.uint8, device="cuda")
    err = torch.empty(nb, dtype=torch.float64, device="cuda")
    gic.encode_device(7, src, n, n, 1, 4, dst, gic.Options(), block_err=err)
    torch.cuda.synchronize()
    blocks = dst.cpu().numpy().reshape(-1, 16)
    e = err.cpu().numpy()
    assert np.isfinite(e).all() and (e >= 0).all()
    low = blocks[:, 0].astype(np.int32)
    assert (low != 0).all()
    modes = np.log2(low & -low).astype(np.int32)          # BC7 mode = lowest set bit
    assert modes.max() <= 5
    dec = oracle_lib.bc7_decode(blocks)                    # (nb, 16, 4)
    img = src.cpu().numpy()[0]
    ref = img.reshape(n // 4, 4, n // 4, 4, 4).transpose(0, 2, 1, 3, 4).reshape(nb, 16, 4)
    d = dec.astype(np.int32) - ref.astype(np.int32)
    mse = float((d * d).sum(dtype=np.int64)) / d.size
    psnr = 10 * np.log10(255.0 ** 2 / mse)
    assert psnr > 40.0, psnr
    row = oracle_lib.encode_image(7, img, first_row=1024, num_rows=1)
    assert np.array_equal(blocks[1024 * (n // 4):1025 * (n // 4)], row)


def _encode_on(stream, fmt, src, w, h, dst, opts=None):
    import torch
    with torch.cuda.stream(stream):
        gic.encode_device(fmt, src, w, h, src.shape[0], src.shape[-1], dst, opts or gic.Options(), stream=stream)


def test_bc7_concurrent_streams_do_not_share_workspace(gpu):
    """Two encodes of different images (each one workspace chunk, <= 65 536
    blocks) in flight at once on two caller streams: both must equal their
    sequential results and sampled rows must equal the oracle (the per-device
    BC7 workspace is serialised on internal lanes, never raced)."""
    import torch
    n = 1024                                   # 65 536 blocks = one chunk
    a = synth.g1_torch(n, n, 1, seed=11, device="cuda")
    b = synth.g1_torch(n, n, 1, seed=12345, device="cuda").flip(2).contiguous()
    nb = (n // 4) ** 2
    seq = [torch.empty(nb * 16, dtype=torch.uint8, device="cuda") for _ in range(2)]
    for src, d in zip((a, b), seq):
        gic.encode_device(7, src, n, n, 1, 4, d, gic.Options())
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    par = [torch.zeros(nb * 16, dtype=torch.uint8, device="cuda") for _ in range(2)]
    _encode_on(s1, 7, a, n, n, par[0])
    _encode_on(s2, 7, b, n, n, par[1])
    torch.cuda.synchronize()
    for k in range(2):
        assert torch.equal(par[k], seq[k]), f"image {k}: concurrent encode differs from the sequential one"
    bx = n // 4
    for k, src in enumerate((a, b)):
        host = src.cpu().numpy()[0]
        ref = oracle_lib.encode_image(7, host, first_row=100, num_rows=1)
        got = par[k].cpu().numpy().reshape(-1, 16)[100 * bx:101 * bx]
        assert np.array_equal(got, ref), _mismatch_report(got, ref)


def test_bc7_multi_slice_stack(gpu):
    """Config 5 shape at reduced size: a stack of G1 slices (slice s seeded
    0x9E3779B9+s, as the batch workload) encoded in one call through the
    block-row shard entry; sampled rows of every slice against the oracle
    under the MSE contract, and bit-identical."""
    import torch
    s, n = 6, 256
    src = synth.g1_torch(n, n, s, seed=0x9E3779B9, device="cuda")
    host = src.cpu().numpy()
    bx = n // 4
    first, rows = 17, 3                       # the same block-row range of every slice
    dst = torch.zeros(s * rows * bx * 16, dtype=torch.uint8, device="cuda")
    gic.encode_device(7, src, n, n, s, 4, dst, gic.Options(), first, rows)
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(s, rows * bx, 16)
    for k in range(s):
        assert np.array_equal(host[k], synth.g1(n, n, seed=0x9E3779B9 + k))
        ref = oracle_lib.encode_image(7, host[k], first_row=first, num_rows=rows)
        check_tolerance(got[k], ref, _src_blocks(host[k], first, rows))
        assert np.array_equal(got[k], ref), (k, _mismatch_report(got[k], ref))


@pytest.mark.parametrize("mask", [0x10, 0x30])
def test_bc7_dual_index_regression_blocks(gpu, mask):
    """The blocks on which the round-1 merged dual-index quantiser build went
    wrong (mode 4 mixes 2- and 3-bit index sets; the cluster count was read
    through a scalar load of lane 0's address): 256 opaque noise
    blocks and 256 G1 blocks, mode 4 (and 4+5) only, every block vs the oracle."""
    for img in (synth.noise_rgba(64, 64, seed=6, alpha=False), synth.g1(64, 64),
                synth.noise_rgba(64, 64, seed=5, alpha=True)):
        blocks = img.reshape(16, 4, 16, 4, 4).transpose(0, 2, 1, 3, 4).reshape(256, 64).astype(np.float32) \
            / np.float32(255.0)
        got = _gpu_blocks_f32(blocks, mask)
        for i, b in enumerate(blocks):
            enc, _ = oracle_lib.bc7_block(b, mask)
            assert got[i].tobytes() == enc, (mask, i)


def test_iteration_cap_hits_are_counted(gpu):
    """the reference's requantisation loop (optQuantAnD_d,
    amd_bc7_3dquant_vpc.cpp:1885-1986; optQuantAnD_f for BC6H) never resets its
    counter, so past its exhaustion it runs until the state is stable.  At the
    default cap a G1 band and an HDR image reach no cap (the output equals the
    oracle's).  With the cap at 0 every BC7 register-quantiser loop stops as
    soon as the reference's counter runs out (blocks that need more
    requantisation passes than its budget of 50): the stops are counted, their
    blocks marked and encoded again through the uncapped general path in the
    same call -- so the output still equals the oracle on every block, and
    gic_last_h4_report names the re-run blocks.  BC6H applies the cap per loop
    and so does its oracle: at cap 0 and cap 3 both stop the same loops and
    the blocks stay bit-identical (the 4000-round fast-forward is exact under
    the cap)."""
    import torch
    img = synth.g1(256, 64)
    hdr = synth.hdr_rgba(256, 256, seed=3)
    src = torch.from_numpy(hdr.reshape(-1).copy()).cuda()
    dst = torch.zeros(64 * 64 * 16, dtype=torch.uint8, device="cuda")
    ref7 = oracle_lib.encode_image_bc7(img, first_row=0, num_rows=4)
    blocks = hdr.reshape(64, 4, 64, 4, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 64)
    gic.iter_cap_hits(reset=True)
    out = gpu_encode(7, img)
    assert gic.iter_cap_hits(reset=True) == 0
    assert gic.last_h4_report() == (0, 0)
    assert np.array_equal(out[:256], ref7)
    gic.encode_device_src(gic.FMT_BC6H, gic.SRC_FLOAT32, src, 256, 256, 1, 4, dst)
    assert gic.iter_cap_hits(reset=True) == 0
    ref6, _ = oracle_lib.bc6h_blocks(blocks)
    assert np.array_equal(dst.cpu().numpy().reshape(-1, 16), ref6)
    hits6 = {}
    gic.set_iter_cap(0)
    try:
        out0 = gpu_encode(7, img)
        hits7 = gic.iter_cap_hits(reset=True)
        rerun, nonterm = gic.last_h4_report()
        for cap in (0, 3):
            gic.set_iter_cap(cap)
            oracle_lib.bc6h_set_cap(cap)
            gic.encode_device_src(gic.FMT_BC6H, gic.SRC_FLOAT32, src, 256, 256, 1, 4, dst)
            hits6[cap] = gic.iter_cap_hits(reset=True)
            ref_c, _ = oracle_lib.bc6h_blocks(blocks)
            got = dst.cpu().numpy().reshape(-1, 16)
            assert np.array_equal(got, ref_c), (cap, int((got != ref_c).any(axis=1).sum()))
    finally:
        gic.set_iter_cap(-1)
        oracle_lib.bc6h_set_cap(-1)
    print(f"\ncap 0: {hits7} BC7 loops stopped, {rerun} blocks re-run, {nonterm} cyclic; BC6H stops {hits6}")
    assert hits7 > 0 and rerun > 0 and nonterm == 0 and hits6[0] > 0
    assert np.array_equal(out0[:256], ref7)        # the re-run blocks are the reference's
    assert np.array_equal(out0, out)
    gpu_encode(7, img[:8])
    assert gic.iter_cap_hits(reset=True) == 0   # the default cap is back
    assert gic.last_h4_report() == (0, 0)
