"""Diagnostic: the linked gather (k_compact_s sums the stripe counts itself, O(stripes^2) reads) against
k_link + the plain gather (KVR_LINK_KERNEL=1), per call on cfg2 (device-resident, manifest on the
device) at several stripe counts (tiles per stripe 128 / 64 / 32 -> 4096 / 8192 / 16384 stripes; past
LINKED_MAX_STRIPES = 8192 the library takes k_link either way).  Prints the median wall time and the
device pipeline time of 15 calls per setting.  Usage: python tools/link_crossover.py"""
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
for tps in (128, 64, 32):
    ctx.set_tiles_per_stripe(tps)
    for link_kernel in (False, True):
        if link_kernel:
            os.environ["KVR_LINK_KERNEL"] = "1"
        else:
            os.environ.pop("KVR_LINK_KERNEL", None)
        walls, pipes, comp = [], [], []
        for it in range(18):
            t = time.perf_counter()
            r = ctx.replay(segs, expected=(man.data_ptr(), n_rec), expected_on_device=True, out_ptr=out.data_ptr(),
                           cap=n_rec + 1024)
            dt = time.perf_counter() - t
            assert r.status == 0 and r.n == n_rec and r.stats.n_crc_fail == 0
            if it >= 3:
                walls.append(dt * 1e3)
                pipes.append(r.stats.ms_total)
                comp.append(r.stats.ms_link + r.stats.ms_compact)
        print(f"stripes {r.stats.n_stripes:6d} {'k_link + gather' if link_kernel else 'linked gather  '}: "
              f"wall {np.median(walls):.3f} ms  pipeline {np.median(pipes):.3f} ms  link+gather {np.median(comp):.3f} ms",
              flush=True)
os.environ.pop("KVR_LINK_KERNEL", None)
ctx.set_tiles_per_stripe(0)
