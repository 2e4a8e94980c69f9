"""world_size-2 gloo test of the multi-GPU path's host logic (CPU): ranks take
contiguous element ranges, compress them independently (the oracle stands
in for the per-rank GPU codec here), all-gather the sizes and derive the
same packing offsets; the sharded archives equal the single-process ones
(a per-element archive is a pure function of its bytes)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.util import float_words

NB = 11  # odd: the last shard is short


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    return [float_words(2, 300 + 517 * i, seed=i) for i in range(NB)]


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dietgpu_fork_amd import dist as D
        from oracle import oracle as O

        xs = _inputs()
        a, b = D.shard_range(NB, rank, world)
        archives = [O.float_compress(xs[i], 2, 10) for i in range(a, b)]
        local = torch.tensor([x.size for x in archives], dtype=torch.int32)
        sizes = D.gather_sizes(local, NB)
        offs = D.archive_offsets(sizes)
        np.save(os.path.join(outdir, f"sizes{rank}.npy"), sizes.numpy())
        np.save(os.path.join(outdir, f"offs{rank}.npy"), offs.numpy())
        for i, arch in zip(range(a, b), archives):
            np.save(os.path.join(outdir, f"arch{i}.npy"), arch)
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_batch():
    from dietgpu_fork_amd import dist as D

    for nb in (0, 1, 7, 8, 256, 8192):
        for world in (1, 2, 4, 8):
            got = [D.shard_range(nb, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == nb
            assert all(got[i][1] == got[i + 1][0] for i in range(world - 1))


def test_two_rank_gloo_size_gather(tmp_path):
    from dietgpu_fork_amd import dist as D
    from oracle import oracle as O

    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    xs = _inputs()
    ref = [O.float_compress(x, 2, 10) for x in xs]
    ref_sizes = np.array([r.size for r in ref], dtype=np.int64)
    for rank in range(2):
        assert np.array_equal(np.load(tmp_path / f"sizes{rank}.npy"), ref_sizes)
        offs = np.load(tmp_path / f"offs{rank}.npy")
        assert np.array_equal(offs, D.archive_offsets(torch.from_numpy(ref_sizes)).numpy())
        assert (offs % 16 == 0).all()
    for i in range(NB):
        assert np.array_equal(np.load(tmp_path / f"arch{i}.npy"), ref[i])


class _OracleCodec:
    """CPU stand-in for dist.GpuFloatCodec in gloo tests (bf16): the oracle's
    float codec, same archives as the GPU path."""

    def compress(self, tensors):
        from oracle import oracle as O

        arch = [O.float_compress(t.view(torch.int16).numpy().view(np.uint16), 2, 10)
                for t in tensors]
        comp = torch.zeros(len(arch), max(a.size for a in arch), dtype=torch.uint8)
        for i, a in enumerate(arch):
            comp[i, : a.size] = torch.from_numpy(a)
        return comp, torch.tensor([a.size for a in arch], dtype=torch.int32)

    def decompress(self, archives, outs):
        from oracle import oracle as O

        for a, o in zip(archives, outs):
            st, words = O.float_decompress(a.numpy(), 2, 10)
            assert st == 0 and words.size == o.numel()
            o.view(torch.int16).copy_(torch.from_numpy(words.view(np.int16)))


def _bf16(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, generator=g) * (1 + seed % 3)).to(torch.bfloat16)


def _gather_inputs(rank):  # k = 3 tensors per rank, sizes differ between ranks
    return [_bf16(n, 10 * rank + i) for i, n in enumerate((1000 + 333 * rank, 5000, 77 * (rank + 1)))]


def _a2a_input(src, dst):
    return _bf16(700 + 1111 * src + 37 * dst, 100 + 10 * src + dst)


def _cc_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dietgpu_fork_amd import dist as D

        got = D.all_gather_compressed(_gather_inputs(rank), codec=_OracleCodec())
        for j, t in enumerate(got):
            np.save(os.path.join(outdir, f"ag{rank}_{j}.npy"), t.view(torch.int16).numpy())
        got = D.all_to_all_compressed([_a2a_input(rank, d) for d in range(world)],
                                      codec=_OracleCodec())
        for s, t in enumerate(got):
            np.save(os.path.join(outdir, f"a2a{rank}_{s}.npy"), t.view(torch.int16).numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_compressed_collectives(tmp_path):
    """all_gather_compressed / all_to_all_compressed deliver every tensor bit
    for bit (world 2, gloo, the oracle codec standing in for the GPU one)."""
    world = 2
    mp.spawn(_cc_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    want = [t for r in range(world) for t in _gather_inputs(r)]
    for rank in range(world):
        for j, t in enumerate(want):
            got = np.load(tmp_path / f"ag{rank}_{j}.npy")
            assert np.array_equal(got, t.view(torch.int16).numpy()), (rank, j)
        for s in range(world):
            got = np.load(tmp_path / f"a2a{rank}_{s}.npy")
            assert np.array_equal(got, _a2a_input(s, rank).view(torch.int16).numpy()), (rank, s)


class _PoisonCodec(_OracleCodec):
    """The oracle codec with one abandoned element on rank 1 (archive size 0,
    as a poisoned compression reports it)."""

    def __init__(self, rank):
        self.rank = rank

    def compress(self, tensors):
        comp, sizes = super().compress(tensors)
        if self.rank == 1:
            sizes[1] = 0
        return comp, sizes


def _poison_worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dietgpu_fork_amd import dist as D

        msgs = []
        for fn, arg in ((D.all_gather_compressed, _gather_inputs(rank)),
                        (D.all_to_all_compressed, [_a2a_input(rank, d) for d in range(world)])):
            try:
                fn(arg, codec=_PoisonCodec(rank))
                msgs.append("no error")
            except RuntimeError as e:
                msgs.append(str(e))
        with open(os.path.join(outdir, f"poison{rank}.txt"), "w") as f:
            f.write("\n".join(msgs))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_abandoned_archive_raises_everywhere(tmp_path):
    """A size-0 (abandoned) archive on one rank makes BOTH collectives raise
    on EVERY rank before the payload exchange (no rank left waiting, no
    zero-length slot aliasing the next archive)."""
    world = 2
    mp.spawn(_poison_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for rank in range(world):
        msgs = (tmp_path / f"poison{rank}.txt").read_text().split("\n")
        assert len(msgs) == 2
        assert "all_gather_compressed" in msgs[0] and "abandoned" in msgs[0], msgs
        assert "all_to_all_compressed" in msgs[1] and "abandoned" in msgs[1], msgs


C5_TOTAL, C5_WORDS = 64, 257  # the c5 plan at test size (bench.py: 8192 x 524288)


def _c5_worker(rank, world, port, outdir):
    """bench.py's N>1 leg minus the GPU: this rank's contiguous share of the
    fixed batch (bench._bf16_rows), compressed locally (oracle standing in for
    the GPU codec), per-element sizes all-gathered, max-over-ranks timing."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from dietgpu_fork_amd import dist as D
        from oracle import oracle as O

        first, last = D.shard_range(C5_TOTAL, rank, world)
        assert last - first == C5_TOTAL // world
        x = bench._bf16_rows(first, last, C5_WORDS, "cpu", chunk=16)
        sizes = torch.tensor([O.float_compress(r.view(torch.int16).numpy().view(np.uint16), 2).size
                              for r in x], dtype=torch.int32)
        allsizes = D.gather_sizes(sizes, C5_TOTAL)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        np.save(os.path.join(outdir, f"c5sizes{rank}.npy"), allsizes.numpy())
        np.save(os.path.join(outdir, f"c5rows{rank}.npy"), x.view(torch.int16).numpy())
        np.save(os.path.join(outdir, f"c5t{rank}.npy"), t.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_c5_sharded_bench_plan(tmp_path, world):
    """Every rank ends with the sizes of the whole fixed batch in element
    order, the shards' rows are the unsharded batch's rows (the data does
    not depend on the sharding), and the timing is the max over ranks."""
    import bench
    from oracle import oracle as O

    mp.spawn(_c5_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    full = bench._bf16_rows(0, C5_TOTAL, C5_WORDS, "cpu", chunk=16)
    ref = np.array([O.float_compress(r.view(torch.int16).numpy().view(np.uint16), 2).size for r in full])
    rows = np.concatenate([np.load(tmp_path / f"c5rows{r}.npy") for r in range(world)])
    assert np.array_equal(rows, full.view(torch.int16).numpy())
    for r in range(world):
        assert np.array_equal(np.load(tmp_path / f"c5sizes{r}.npy"), ref)
        assert float(np.load(tmp_path / f"c5t{r}.npy")[0]) == world


def test_pack_matches_per_element_copies():
    from dietgpu_fork_amd import dist as D

    g = torch.Generator().manual_seed(3)
    comp = torch.randint(0, 256, (7, 100), generator=g, dtype=torch.uint8)
    sizes = torch.tensor([0, 1, 15, 16, 17, 99, 100])
    offs = D.archive_offsets(sizes)
    length = int(offs[-1] + (sizes[-1] + 15) // 16 * 16) + 5
    buf = D._pack(comp, sizes, offs, length, "cpu")
    assert buf.numel() == length
    for i in range(7):
        o, s = int(offs[i]), int(sizes[i])
        assert torch.equal(buf[o:o + s], comp[i, :s])
