"""Host memory costs on the GPU box for the open path: pinned allocation (one 4-GiB
kvr_host_alloc vs 16 concurrent 256-MiB ones) and first-touch of pageable memory (1 vs 16
threads).  Prints one line per case."""
import ctypes as C
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-kvstore-v2_amd"))
import kvreplay as K

rep, _ = K.native()
G = 1 << 30
TOT = 4 * G


def alloc(n):
    p = C.c_void_p()
    rc = rep.kvr_host_alloc(n, C.byref(p))
    assert rc == 0
    return p.value


for rnd in range(2):
    t = time.perf_counter()
    p = alloc(TOT)
    a1 = time.perf_counter() - t
    rep.kvr_host_free(p)
    for nt in (4, 16):
        t = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            ps = list(ex.map(alloc, [TOT // nt] * nt))
        an = time.perf_counter() - t
        t = time.perf_counter()
        for q in ps:
            rep.kvr_host_free(q)
        fr = time.perf_counter() - t
        print(f"round {rnd}: pinned 1 x 4 GiB {a1*1e3:.1f} ms | {nt} x {4096//nt} MiB concurrent {an*1e3:.1f} ms "
              f"(free {fr*1e3:.1f} ms)", flush=True)
    for nt in (1, 16):
        t = time.perf_counter()
        a = np.empty(TOT, dtype=np.uint8)
        step = TOT // nt
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(lambda i: a[i * step:(i + 1) * step].fill(1), range(nt)))
        tt = time.perf_counter() - t
        del a
        print(f"round {rnd}: pageable 4 GiB first touch, {nt} threads {tt*1e3:.1f} ms", flush=True)
