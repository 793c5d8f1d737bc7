"""Diagnostic: k_replay time against the stripe length (tiles per stripe) on a bench config.
  python tools/tps_sweep.py [cfg2|cfg3|cfg5] [n_segments] tps1 tps2 ...   (0 = automatic)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kvstore-v2_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvreplay as K  # noqa: E402
from bench import CONFIGS  # noqa: E402

cfg = sys.argv[1]
nseg, seg_bytes, kw, desc = CONFIGS[cfg]
if int(sys.argv[2]):
    nseg = int(sys.argv[2])
spec = K.GenSpec(seed=0x6B767265706C6179 + int(cfg[3:]), seg_bytes=seg_bytes, **kw)
ctx = K.Context(0)
sizes = [K.gen_segment_size(spec, s) for s in range(nseg)]
offs, tot = [], 0
for ln, _ in sizes:
    offs.append(tot)
    tot += (ln + 255) & ~255
n_rec = sum(nr for _, nr in sizes)
data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda:0")
for s, (ln, nr), o in zip(range(nseg), sizes, offs):
    ctx.gen_segment_device(spec, s, data.data_ptr() + o, ln, None, 0)
torch.cuda.synchronize()
segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
out = torch.empty((n_rec + 1024) * 32, dtype=torch.uint8, device="cuda:0")
for tps in [int(x) for x in sys.argv[3:]]:
    ctx.set_tiles_per_stripe(tps)
    ms = []
    for i in range(8):
        r = ctx.replay(segs, on_device=True, out_ptr=out.data_ptr(), cap=n_rec + 1024)
        assert r.status == 0 and r.n == n_rec
        if i >= 2:
            ms.append((r.stats.ms_replay, r.stats.ms_total, r.stats.n_stripes, r.stats.n_redo))
    a = np.array(ms)
    print(f"{cfg} tps={tps}: k_replay {a[:, 0].mean():.4f} ms, pipeline {a[:, 1].mean():.4f} ms, "
          f"stripes {int(a[0, 2])}, redo {int(a[0, 3])}", flush=True)
