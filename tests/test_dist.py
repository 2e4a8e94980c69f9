"""world_size-2 gloo test of the multi-GPU path's host logic (CPU): ranks take
contiguous element ranges, compress them independently (the oracle stands
in for the per-rank GPU codec here), all-gather the sizes and derive the
same packing offsets; the sharded archives equal the single-process ones
(a per-element archive is a pure function of its bytes)."""
import os
import socket

import numpy as np
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
