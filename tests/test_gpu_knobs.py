"""k_compress's generation-scheduling knobs (DIETGPU_COMPRESS_PREFETCH,
DIETGPU_COMPRESS_STAGGER; off by default) must not change a
byte of the archives.  The library reads them once per process, so the
compression runs in a child process on a batch of several generations of
workgroups (c2's shape); archives are compared with the oracle here."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys
    import numpy as np
    import torch
    sys.path.insert(0, {root!r})
    import dietgpu_fork_amd  # noqa: F401
    from dietgpu_fork_amd import codec as C
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(256, 524288, generator=g, device="cuda").to(torch.bfloat16)
    arch, sizes = C.float_compress_stride(x, ws=C.Workspace(768 << 20))
    sizes = sizes.cpu().numpy()
    pick = [0, 1, 77, 128, 255]
    np.savez({out!r}, x=x[pick].view(torch.int16).cpu().numpy(), sizes=sizes[pick],
             arch=np.stack([arch[i, : sizes.max()].cpu().numpy() for i in pick]))
""")


@pytest.mark.parametrize("knobs", [{"DIETGPU_COMPRESS_PREFETCH": "1"},
                                   {"DIETGPU_COMPRESS_STAGGER": "500"}])
def test_scheduling_knobs_keep_archives(tmp_path, knobs):
    out = str(tmp_path / "r.npz")
    env = dict(os.environ, **knobs)
    subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, out=out)], env=env, check=True,
                   timeout=120)
    r = np.load(out)
    for i in range(len(r["sizes"])):
        ref = O.float_compress(r["x"][i].view(np.uint16), 2)
        assert int(r["sizes"][i]) == ref.size
        np.testing.assert_array_equal(r["arch"][i, : ref.size], ref)
