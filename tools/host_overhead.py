"""Diagnostic: where a kvr_replay call's wall time goes beyond its device pipeline (cfg2, device-resident).
Prints per-call wall (Python wrapper, and a bare ctypes call), the pipeline's event time (ev0 -> ev3:
k_replay, k_link, k_compact_s) and the difference."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kvstore-v2_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import kvreplay as K  # noqa: E402
from bench import CONFIGS  # noqa: E402

nseg, seg_bytes, kw, _ = CONFIGS["cfg2"]
spec = K.GenSpec(seed=0x6B767265706C6179 + 2, seg_bytes=seg_bytes, **kw)
ctx = K.Context(0)
sizes = [K.gen_segment_size(spec, s) for s in range(nseg)]
offs, tot = [], 0
for ln, _ in sizes:
    offs.append(tot)
    tot += (ln + 255) & ~255
n_rec = sum(nr for _, nr in sizes)
data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda")
man = torch.empty(n_rec + 1, dtype=torch.int32, device="cuda")
eo = 0
for s, (ln, nr), o in zip(range(nseg), sizes, offs):
    ctx.gen_segment_device(spec, s, data.data_ptr() + o, ln, man.data_ptr() + 4 * eo, nr)
    eo += nr
torch.cuda.synchronize()
segs = K.SegmentList([(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)], seg_ids=list(range(nseg)),
                     on_device=True)
out = torch.empty((n_rec + 1024) * 32, dtype=torch.uint8, device="cuda")
for _ in range(5):
    ctx.replay(segs, expected=(man.data_ptr(), n_rec), expected_on_device=True, out_ptr=out.data_ptr(), cap=n_rec + 1024)
walls, pipes = [], []
for _ in range(30):
    t = time.perf_counter()
    r = ctx.replay(segs, expected=(man.data_ptr(), n_rec), expected_on_device=True, out_ptr=out.data_ptr(), cap=n_rec + 1024)
    walls.append(time.perf_counter() - t)
    pipes.append(r.stats.ms_total)
rep = ctx._rep
flags = K.SEGS_ON_DEVICE | K.OUT_ON_DEVICE | K.EXPECTED_ON_DEVICE
n_out, err = C.c_size_t(), K.Error()
bare = []
for _ in range(30):
    t = time.perf_counter()
    rc = rep.kvr_replay(ctx.h, segs.arr, segs.n, flags, man.data_ptr(), n_rec, out.data_ptr(), n_rec + 1024,
                        C.byref(n_out), C.byref(err))
    bare.append(time.perf_counter() - t)
    assert rc == 0
w, b, p = np.median(walls) * 1e3, np.median(bare) * 1e3, np.median(pipes)
print(f"per call (median of 30): wrapper wall {w:.3f} ms, bare ctypes wall {b:.3f} ms, device pipeline "
      f"(ev0->ev3) {p:.3f} ms; host + tail {b - p:.3f} ms, wrapper {w - b:.3f} ms")
