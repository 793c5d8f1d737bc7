"""Diagnostic: kernel time of k_replay with parts switched off (-DKVR_ABLATE=mask builds under
lib/ablate/).  The results are wrong by design; only the time matters.
  python tools/ablate.py [cfg2|cfg3|cfg5] [n_segments] [mask]   (one mask per process: the HIP
  runtime registers kernels by name, so two libraries in one process may launch the same code)"""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mini-kvstore-v2_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import kvreplay as K  # noqa: E402
from bench import CONFIGS  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
nseg_o = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ABL = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "ablate")
nseg, seg_bytes, kw, desc = CONFIGS["cfg3" if cfg == "etag" else cfg]
if nseg_o:
    nseg = nseg_o
spec = None if cfg == "etag" else K.GenSpec(seed=0x6B767265706C6179 + int(cfg[3:]), seg_bytes=seg_bytes, **kw)
P, U32, U64, SZ = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t
VAR = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "variants")
AB = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "ab")
if len(sys.argv) > 3:   # a mask (lib/ablate) or a variant name (lib/variants, build.py VARIANTS)
    masks = [int(sys.argv[3]) if sys.argv[3].isdigit() else sys.argv[3]]
else:
    masks = sorted(int(f[len("libkvreplay_a"):-3]) for f in os.listdir(ABL) if f.startswith("libkvreplay_a"))
for mask in masks:
    path = os.path.join(ABL, f"libkvreplay_a{mask}.so") if isinstance(mask, int) else os.path.join(VAR, f"libkvreplay_{mask}.so")
    if not isinstance(mask, int) and os.path.exists(os.path.join(AB, f"libkvreplay_{mask}.so")):
        path = os.path.join(AB, f"libkvreplay_{mask}.so")   # an A/B build (tools/build_ab.sh)
    vp = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "vpair", str(mask), "libkvreplay.so")
    if not isinstance(mask, int) and os.path.exists(vp):
        path = vp   # a variant pair (build.py build_variant_pair)
    if mask == "main":   # the shipped library itself
        path = os.path.join(ROOT, "mini-kvstore-v2_amd", "lib", "libkvreplay.so")
    lib = C.CDLL(path)   # the only kvreplay library in this process
    lib.kvr_ctx_create.argtypes = [C.c_int, C.POINTER(P)]
    lib.kvr_replay.argtypes = [P, C.POINTER(K.Segment), SZ, U32, P, SZ, P, SZ, C.POINTER(SZ), C.POINTER(K.Error)]
    lib.kvr_last_stats.argtypes = [P, C.POINTER(K.Stats)]
    lib.kvr_gen_segment_device.argtypes = [P, C.POINTER(K.GenParams), U64, P, U64, C.POINTER(U64), P, U64,
                                           C.POINTER(U64)]
    h = P()
    assert lib.kvr_ctx_create(0, C.byref(h)) == 0
    if cfg == "etag":   # k_etag_chunk on bench.py --mode etag's workload: 131072 x 64-KiB blobs in HBM
        import numpy as np
        n_blob, blob = 131072, 65536
        g = torch.Generator(device="cuda")
        g.manual_seed(0x6B767265)
        data = torch.randint(0, 256, (n_blob * blob,), dtype=torch.uint8, device="cuda", generator=g)
        torch.cuda.synchronize()
        offs = np.arange(n_blob, dtype=np.uint64) * blob
        lens = np.full(n_blob, blob, dtype=np.uint64)
        out = np.zeros(n_blob, dtype=np.uint32)
        nf = U64()
        lib.kvr_etag_batch.argtypes = [P, P, U64, P, P, SZ, U32, P, P, C.POINTER(U64)]
        lib.kvr_last_etag_stats.argtypes = [P, C.POINTER(K.EtagStats)]
        ms = []
        for it in range(12):
            rc = lib.kvr_etag_batch(h, data.data_ptr(), data.numel(), offs.ctypes.data, lens.ctypes.data, n_blob,
                                    K.SEGS_ON_DEVICE, None, out.ctypes.data, C.byref(nf))
            st = K.EtagStats()
            lib.kvr_last_etag_stats(h, C.byref(st))
            ms.append(st.ms_chunk)
        import zlib
        ok = all(int(out[i]) == zlib.crc32(data[i * blob:(i + 1) * blob].cpu().numpy().tobytes()) for i in (0, 77, n_blob - 1))
        t = min(ms[1:])
        med = sorted(ms[1:])[len(ms[1:]) // 2]
        print(f"etag build={mask!s:>6}: rc={rc} crc_ok={ok} k_etag_chunk {t:.3f} ms (median {med:.3f})  "
              f"{n_blob * blob / t / 1e6:.1f} GB/s frac {n_blob * blob / t / 1e6 / 8000:.3f}", flush=True)
        continue
    gp = spec.c()
    sizes = []
    for s in range(nseg):
        ln, nr = U64(), U64()
        lib.kvr_gen_segment_device(h, C.byref(gp), s, None, 0, C.byref(ln), None, 0, C.byref(nr))
        sizes.append((ln.value, nr.value))
    offs, tot = [], 0
    for ln, _ in sizes:
        offs.append(tot)
        tot += (ln + 255) & ~255
    nrec = sum(n for _, n in sizes)
    data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda")
    for s, (ln, nr) in enumerate(sizes):
        ln2, nr2 = U64(), U64()
        assert lib.kvr_gen_segment_device(h, C.byref(gp), s, data.data_ptr() + offs[s], ln, C.byref(ln2), None, 0,
                                          C.byref(nr2)) == 0
    torch.cuda.synchronize()
    segs = (K.Segment * nseg)(*[K.Segment(s, data.data_ptr() + o, ln) for s, ((ln, _), o) in enumerate(zip(sizes, offs))])
    out = torch.empty((nrec * 4 + 4096) * 32, dtype=torch.uint8, device="cuda")
    ms = []
    for it in range(12):
        n = SZ()
        e = K.Error()
        rc = lib.kvr_replay(h, segs, nseg, K.SEGS_ON_DEVICE | K.OUT_ON_DEVICE, None, 0, out.data_ptr(), nrec * 4 + 4096,
                            C.byref(n), C.byref(e))
        st = K.Stats()
        lib.kvr_last_stats(h, C.byref(st))
        ms.append(st.ms_replay)
    t = max(min(ms[1:]), 1e-9)
    med = sorted(ms[1:])[len(ms[1:]) // 2]
    print(f"{cfg} ablate={mask!s:>6} (1 records, 2 value CRC, 4 hops): rc={rc} n={n.value}/{nrec} k_replay {t:.3f} ms"
          f" (median {med:.3f})  {tot / t / 1e6:.1f} GB/s  seg_bytes={sum(ln for ln, _ in sizes)}", flush=True)
