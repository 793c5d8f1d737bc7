"""Diagnostic: per-phase cycle breakdown of k_replay's tile loop (build with -DKVR_PROF into
lib/libkvreplay_prof.so).  Usage: python tools/prof_phases.py [cfg2|cfg3|...] [n_segments]
(k_piece's phases when it ran; KVR_NO_PIECE=1 for k_replay's tile loop)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kvstore-v2_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import kvreplay as K  # noqa: E402
from bench import CONFIGS  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
nseg_override = int(sys.argv[2]) if len(sys.argv) > 2 else 0
lib = C.CDLL(os.environ.get("KVR_PROF_LIB") or os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "libkvreplay_prof.so"))
P, U64, U32, SZ = C.c_void_p, C.c_uint64, C.c_uint32, C.c_size_t
lib.kvr_ctx_create.argtypes = [C.c_int, C.POINTER(P)]
lib.kvr_replay.argtypes = [P, C.POINTER(K.Segment), SZ, U32, P, SZ, P, SZ, C.POINTER(SZ), C.POINTER(K.Error)]
lib.kvr_gen_segment_device.argtypes = [P, C.POINTER(K.GenParams), U64, P, U64, C.POINTER(U64), P, U64, C.POINTER(U64)]
lib.kvr_last_stats.argtypes = [P, C.POINTER(K.Stats)]
lib.kvr_prof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]

nseg, seg_bytes, kw, desc = CONFIGS[cfg]
if nseg_override:
    nseg = nseg_override
spec = K.GenSpec(seed=0x6B767265706C6179 + int(cfg[3:]), seg_bytes=seg_bytes, **kw).c()
ctx = P()
assert lib.kvr_ctx_create(0, C.byref(ctx)) == 0
sizes = []
for s in range(nseg):
    ln, nr = U64(), U64()
    lib.kvr_gen_segment_device(ctx, C.byref(spec), s, None, 0, C.byref(ln), None, 0, C.byref(nr))
    sizes.append((ln.value, nr.value))
offs, tot = [], 0
for ln, _ in sizes:
    offs.append(tot)
    tot += (ln + 255) & ~255
nrec = sum(n for _, n in sizes)
data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda")
for s, (ln, nr), o in zip(range(nseg), sizes, offs):
    ln2, nr2 = U64(), U64()
    assert lib.kvr_gen_segment_device(ctx, C.byref(spec), s, data.data_ptr() + o, ln, C.byref(ln2), None, 0,
                                      C.byref(nr2)) == 0
torch.cuda.synchronize()
segs = (K.Segment * nseg)(*[K.Segment(s, data.data_ptr() + o, ln) for s, ((ln, _), o) in enumerate(zip(sizes, offs))])
out = torch.empty((nrec + 1024) * 32, dtype=torch.uint8, device="cuda")
prof = (C.c_ulonglong * 16)()
for it in range(3):
    lib.kvr_prof_read(prof, 1)
    n = SZ()
    e = K.Error()
    rc = lib.kvr_replay(ctx, segs, nseg, K.SEGS_ON_DEVICE | K.OUT_ON_DEVICE, None, 0, out.data_ptr(), nrec + 1024,
                        C.byref(n), C.byref(e))
    st = K.Stats()
    lib.kvr_last_stats(ctx, C.byref(st))
    lib.kvr_prof_read(prof, 0)
def stripe_spread():
    """k_piece / k_replay per-stripe (start, end, HW_ID, XCC_ID) from the diagnostic build."""
    ns = min(st.n_stripes, 16384)
    pst = (C.c_ulonglong * (4 * ns))()
    lib.kvr_prof_stripes.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    if lib.kvr_prof_stripes(pst, ns) == 0:
        import numpy as np
        a = np.frombuffer(pst, dtype=np.uint64).reshape(ns, 4).astype(np.int64)
        t0 = a[:, 0].min()
        beg, end = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0
        dur = end - beg
        hw = a[:, 2]
        wave, simd, cu, se = hw & 15, (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 13) & 7
        xcc = a[:, 3] & 15
        q = np.percentile(dur, [0, 10, 50, 90, 100])
        print(f"  stripe us: start max {beg.max():.1f}; duration min/p10/p50/p90/max "
              + " ".join(f"{v:.0f}" for v in q) + f"; end p50 {np.median(end):.0f} max {end.max():.0f}")
        wl = np.arange(ns) % 16
        print("  mean duration by wave of the workgroup: " + " ".join(f"{dur[wl == i].mean():.0f}" for i in range(16)))
        print("  mean duration by XCC: " + " ".join(f"{dur[xcc == i].mean():.0f}" for i in range(8) if (xcc == i).any()))
        print("  mean duration by SIMD: " + " ".join(f"{dur[simd == i].mean():.0f}" for i in range(4)))
        # per CU (xcc, se, cu): the spread of CU means, and of the spread inside a CU
        key = (xcc * 8 + se) * 16 + cu
        cus = np.unique(key)
        cm = np.array([dur[key == k].mean() for k in cus])
        cs = np.array([dur[key == k].max() - dur[key == k].min() for k in cus])
        print(f"  CUs {len(cus)}: CU-mean duration min/p50/max {cm.min():.0f} {np.median(cm):.0f} {cm.max():.0f}; "
              f"in-CU max-min p50 {np.median(cs):.0f} max {cs.max():.0f}")


# KVR_STAMP slots of kvr_replay_kernel.hip (unused slots print 0)
if os.environ.get("KVR_NO_PIECE") is None and st.n_tiles and prof[6]:   # k_piece's slots (kvr_replay_kernel.hip KVR_PSTAMP)
    steps, flushes = prof[6], prof[7]
    tot_c = sum(prof[i] for i in (0, 1, 2, 3, 4, 5, 8, 9))
    print(f"{cfg} (k_piece): rc={rc} n={n.value}/{nrec} stripes={st.n_stripes} ms_replay={st.ms_replay:.3f} "
          f"steps={steps} flushes={flushes}")
    for i, nm in [(0, "setup (search, prediction)"), (8, "window merge (wait)"), (4, "flush"), (9, "window issue"),
                  (1, "crc_step (incl. load wait)"), (2, "issue"), (3, "finish_step"), (5, "close")]:
        print(f"  {nm:28s} {prof[i] / steps:10.0f} cycles/step  {100 * prof[i] / max(tot_c, 1):5.1f}%")
    print(f"  total {tot_c / steps:10.0f} cycles/step (per wave, lane 0); {tot_c / st.n_stripes:.0f} cycles/stripe")
    if prof[12]:   # s_memrealtime (100 MHz) over the same stretches, and the span of all k_piece waves
        span = (prof[13] - (~prof[14] & (2**64 - 1))) / 100.0
        print(f"  clock {tot_c / prof[12] * 100:.0f} MHz (s_memtime / s_memrealtime); stripe mean "
              f"{prof[12] / st.n_stripes / 100:.1f} us; first wave start to last wave end {span:.1f} us")
    stripe_spread()
    sys.exit(0)
names = ["setup(load)", "stride-decode", "hop-loop+rest", "finalize", "bookkeep", "wait(vmcnt)", "stride-emit",
         "cand-swar", "crc-entry", "unit-loop+kmul", "scan", "cand-decode", "cand-walk", "cand-emit", "spec tiles", "batched tiles"]
tiles = st.n_tiles
tot_c = sum(prof[i] for i in range(14))   # (slots 14, 15: tile counts, KVR_PROF builds)
print(f"{cfg}: rc={rc} n={n.value}/{nrec} bytes={tot} tiles={tiles} stripes={st.n_stripes} ms_replay={st.ms_replay:.3f}"
      f" GB/s={tot / st.ms_replay / 1e6:.1f}")
for i, nm in enumerate(names):
    if i >= 14:
        print(f"  {nm:10s} {prof[i] / tiles:10.3f} of the tiles")
        continue
    print(f"  {nm:10s} {prof[i] / tiles:10.0f} cycles/tile  {100 * prof[i] / max(tot_c, 1):5.1f}%")
print(f"  total      {tot_c / tiles:10.0f} cycles/tile (wave-0 lane-0 view)")
stripe_spread()
