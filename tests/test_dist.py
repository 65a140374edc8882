"""Multi-rank block-row sharding on CPU (gloo, world size 2).

Each rank encodes its shard of a 2-slice image whose block-row count does not
divide evenly (contiguous and interleaved row chunks), the shards are gathered
to rank 0 and reassembled, and the result must equal the single-process encode
byte for byte.  The per-shard encoder here is
the CPU checker (oracle) with the product encoder's signature: this test covers
the sharding, padding, gather and reassembly logic that bench.py and the
multi-GPU path use; the HIP encoder itself is covered by the -m gpu tests.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gfx_imagecompress_amd import shard
from gfx_imagecompress_amd import synth

FMT_CASES = [(1, 4), (5, 2), (7, 4)]


def test_shard_rows_partition():
    for by in range(0, 40):
        for world in range(1, 9):
            spans = [shard.shard_rows(by, world, r) for r in range(world)]
            assert sum(n for _, n in spans) == by
            pos = 0
            for first, n in spans:
                assert first == pos
                pos += n
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1
    with pytest.raises(ValueError):
        shard.shard_rows(4, 2, 2)


def test_row_ranges_partition():
    """Contiguous and interleaved assignments cover every block row exactly once."""
    for by in range(0, 70):
        for world in range(1, 9):
            for chunk in (0, 1, 3, 16):
                seen = []
                for r in range(world):
                    rr = shard.row_ranges(by, world, r, chunk)
                    for first, n in rr:
                        assert n > 0 and (chunk == 0 or world == 1 or n <= chunk)
                        seen.extend(range(first, first + n))
                    assert shard.shard_blocks(by, 5, 2, world, r, chunk) == sum(n for _, n in rr) * 10
                assert sorted(seen) == list(range(by))
    assert shard.row_ranges(40, 4, 1, 4) == [(4, 4), (20, 4), (36, 4)]
    assert shard.row_ranges(10, 2, 1, 4) == [(4, 4)]
    assert shard.row_ranges(10, 2, 0, 4) == [(0, 4), (8, 2)]
    assert shard.row_ranges(10, 1, 0, 4) == [(0, 10)]   # one rank: one range


def _oracle_encoder(fmt, src, width, height, slices, channels, dst, options, first_block_row, num_block_rows,
                    stream=None):
    import oracle_lib
    img = src.numpy().reshape(slices, height, width, channels)
    out = oracle_lib.encode_image(fmt, img, bc4_channel=0, first_row=first_block_row, num_rows=num_block_rows,
                                  threads=2)
    dst[: out.size] = torch.from_numpy(out.reshape(-1))


def _image(fmt, ch):
    w, h, s = 36, 18, 2        # 9 x 5 blocks per slice: shards of 3 and 2 rows
    sl = [synth.noise_rgba(w, h, seed=11 + i, alpha=(fmt == 7 and i == 1))[..., :ch] for i in range(s)]
    return np.ascontiguousarray(np.stack(sl)), w, h, s


def _bench_worker(rank, world, port, q):
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        t = bench._max_over_ranks(torch.tensor([1.0 + rank, 10.0 - rank], dtype=torch.float64), world)
        g = bench._gather_root(torch.full((5,), rank + 1, dtype=torch.uint8), world)
        spread = bench._spread_over_ranks(3.0 + rank, world)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, (t.tolist(), None if g is None else g.tolist(), spread)))
    except Exception as e:   # pragma: no cover
        q.put((rank, repr(e)))


def test_bench_reductions_two_ranks():
    """bench.py's max-over-ranks timing reduction and bitstream gather (gloo path)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
        t, g, spread = got[r]
        assert t == [2.0, 10.0]
        assert spread == [3.0, 4.0]
        # gather to the root only
        assert g == ([1] * 5 + [2] * 5 if r == 0 else None)


def _worker(rank, world, port, q):
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = []
        for fmt, ch in FMT_CASES:
            img, w, h, s = _image(fmt, ch)
            src = torch.from_numpy(img.reshape(-1))
            for chunk in (0, 1, 2):
                local = shard.encode_shard(fmt, src, w, h, s, ch, rank, world, encoder=_oracle_encoder, chunk=chunk)
                full = shard.gather_to_root(local, fmt, w, h, s, world, chunk=chunk)
                res.append((fmt, chunk, None if full is None else full.numpy().tobytes(), local.numel()))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:   # pragma: no cover - reported by the parent
        q.put((rank, repr(e)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_shards_reassemble_to_single_process_encode():
    import oracle_lib
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
    for i, (fmt, ch) in enumerate(FMT_CASES):
        img, w, h, s = _image(fmt, ch)
        ref = oracle_lib.encode_image(fmt, img, bc4_channel=0, threads=2).reshape(-1).tobytes()
        bb = 8 if fmt == 1 else 16
        # rows per rank: contiguous 3 + 2; chunks of 1 -> {0,2,4} + {1,3}; chunks of 2 -> {0,1,4} + {2,3}
        for j, chunk in enumerate((0, 1, 2)):
            fmt0, chunk0, full0, n0 = got[0][3 * i + j]
            fmt1, chunk1, full1, n1 = got[1][3 * i + j]
            assert (fmt0, chunk0) == (fmt, chunk) == (fmt1, chunk1)
            assert full0 == ref, (fmt, chunk)      # reassembled on the root
            assert full1 is None                   # gather to the root only
            assert n0 == 3 * 9 * 2 * bb and n1 == 2 * 9 * 2 * bb


def _split_worker(rank, world, port, q):
    """bench.py's 8K split: rank r encodes block rows shard_rows(BY, N, r) of the
    ONE texture into its RootGather buffer, one gather to rank 0 per step."""
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        import oracle_lib
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = []
        for fmt, size in ((1, 64), (1, 52), (5, 40)):
            ch = 4 if fmt == 1 else 2
            img = synth.g1(size, size)[..., :ch] if fmt == 1 else synth.noise_rgba(size, size, seed=5)[..., :2]
            img = np.ascontiguousarray(img)
            by = bx = (size + 3) // 4
            split = bench.Split(by, world, rank, weak=False)
            g = bench.RootGather(split, bx, 8 if fmt == 1 else 16, "cpu")
            out = oracle_lib.encode_image(fmt, img, bc4_channel=0, first_row=split.first, num_rows=split.rows,
                                          threads=2).reshape(-1)
            for _ in range(3):      # three timed steps: encode into this step's target, gather it
                g.local[: out.size] = torch.from_numpy(out)   # (asynchronously; the targets alternate)
                g()
            res.append((fmt, size, split.first, split.rows, None if rank else g.image_host().tobytes()))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:   # pragma: no cover
        q.put((rank, repr(e)))


def test_bench_8k_split_reassembles_one_image():
    """The strong-scaling split of bench.py's 8K workload (reduced sizes, one of
    them not a multiple of the rank count): the gathered image on rank 0 equals
    the single-process encode byte for byte; rank 1 receives nothing."""
    import oracle_lib
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
    for i, (fmt, size) in enumerate(((1, 64), (1, 52), (5, 40))):
        ch = 4 if fmt == 1 else 2
        img = synth.g1(size, size)[..., :ch] if fmt == 1 else synth.noise_rgba(size, size, seed=5)[..., :2]
        ref = oracle_lib.encode_image(fmt, np.ascontiguousarray(img), bc4_channel=0, threads=2).tobytes()
        by = (size + 3) // 4
        f0, s0, first0, rows0, img0 = got[0][i]
        f1, s1, first1, rows1, img1 = got[1][i]
        assert (first0, rows0, first1, rows1) == (0, (by + 1) // 2, (by + 1) // 2, by // 2)
        assert img0 == ref and img1 is None


def test_bench_gpus_flag_launches_ranks(monkeypatch):
    """bench.py --gpus N outside torchrun starts N ranks as a child
    torch.distributed.run (no exec, before any GPU call); under torchrun a
    WORLD_SIZE that disagrees with --gpus is an error, not a silent N=1 run."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", lambda cmd: seen.setdefault("cmd", cmd) and 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    args = bench.parse()
    assert bench.relaunch_if_needed(args) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.relaunch_if_needed(bench.parse()) is None          # N=1 runs in-process
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    assert bench.relaunch_if_needed(bench.parse()) is None          # torchrun rank
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8"])
    with pytest.raises(SystemExit):
        bench.relaunch_if_needed(bench.parse())


def test_c_abi_multi_split_matches_shard_rows():
    """gic_encode_multi's split of the slice-major block rows (the C ABI's
    multi-GPU path, gic_multi.cpp) is shard.shard_rows: the same contiguous
    ranges bench.py and the torch.distributed path use.  Host-only, no GPU."""
    import gfx_imagecompress_amd as gic
    for rows in list(range(0, 70)) + [2048, 2048 * 64, 1024 * 64 + 5]:
        for n in range(1, 9):
            assert [gic.multi_split(rows, n, i) for i in range(n)] == [shard.shard_rows(rows, n, i) for i in range(n)]
