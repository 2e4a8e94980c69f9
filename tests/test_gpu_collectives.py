"""Compressed collectives (dietgpu_fork_amd/dist.py) over RCCL on one GPU:
world_size 1 with the "nccl" backend runs the real GPU codec (k_pcompress or
k_hist -> k_encode, k_decode) and the real RCCL calls; the gloo world-2 test in test_dist.py
covers the multi-rank bookkeeping on the CPU."""
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pg():
    import dietgpu_fork_amd  # noqa: F401

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _bf16(n, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(n, generator=g) * (1 + seed % 4)).to(torch.bfloat16).cuda()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_all_gather_compressed_rccl(pg, dtype):
    from dietgpu_fork_amd import dist as D

    xs = [_bf16(n, i).to(dtype) for i, n in enumerate((1, 4095, 65536, 300001))]
    got = D.all_gather_compressed(xs)
    assert len(got) == len(xs)
    for x, y in zip(xs, got):
        assert y.dtype == dtype and torch.equal(y, x)


def test_all_to_all_compressed_rccl(pg):
    from dietgpu_fork_amd import dist as D

    x = _bf16(123457, 9)
    (y,) = D.all_to_all_compressed([x])
    assert torch.equal(y, x)
