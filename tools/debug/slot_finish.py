"""Per-dispatch-slot finish times of k_pcompress workgroups from the last
stamps3 run (gpurun_out/stamps3.npy): slot = blockIdx / 256 (4 workgroups
per CU, round-robin dispatch)."""
import os
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
h = np.load(os.path.join(ROOT, "gpurun_out", "stamps3.npy"))
st = h.reshape(4096, 8, 4, 16).astype(np.float64)
t0 = st[st > 0].min()
us = np.where(st > 0, (st - t0) / 100.0, np.nan)
fin = np.nanmax(us[:1024, :, 0, 9], axis=1)
slot = np.arange(1024) // 256
print("span %.1f us; finish by slot median" % np.nanmax(us),
      [round(float(np.nanmedian(fin[slot == s])), 1) for s in range(4)],
      "max", [round(float(np.nanmax(fin[slot == s])), 1) for s in range(4)])
