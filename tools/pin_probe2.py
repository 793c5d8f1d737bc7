"""Pageable vs registered host memory for the open path's transfers (4 GiB): H2D from pageable
memory (HIP's own staging), hipHostRegister cost, H2D from registered memory."""
import ctypes as C
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
G = 1 << 30
TOT = 4 * G
d = torch.empty(TOT, dtype=torch.uint8, device="cuda")
for rnd in range(2):
    a = np.empty(TOT, dtype=np.uint8)
    step = TOT // 16
    with ThreadPoolExecutor(16) as ex:
        list(ex.map(lambda i: a[i * step:(i + 1) * step].fill(1), range(16)))
    t = torch.from_numpy(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(t)
    torch.cuda.synchronize()
    pg = time.perf_counter() - t0
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(a.ctypes.data, TOT, 0)
    reg = time.perf_counter() - t0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d.copy_(t, non_blocking=True)
    torch.cuda.synchronize()
    rg = time.perf_counter() - t0
    t0 = time.perf_counter()
    hip.hipHostUnregister(a.ctypes.data)
    unreg = time.perf_counter() - t0
    # register in 16 concurrent 256-MiB pieces
    t0 = time.perf_counter()
    with ThreadPoolExecutor(16) as ex:
        rcs = list(ex.map(lambda i: hip.hipHostRegister(a.ctypes.data + i * step, step, 0), range(16)))
    reg16 = time.perf_counter() - t0
    for i in range(16):
        hip.hipHostUnregister(a.ctypes.data + i * step)
    print(f"round {rnd}: pageable H2D 4 GiB {pg*1e3:.1f} ms ({TOT/pg/2**30:.1f} GiB/s) | hipHostRegister rc={rc} "
          f"{reg*1e3:.1f} ms, 16 pieces concurrent {reg16*1e3:.1f} ms (rcs {set(rcs)}) | H2D registered {rg*1e3:.1f} ms "
          f"({TOT/rg/2**30:.1f} GiB/s) | unregister {unreg*1e3:.1f} ms", flush=True)
    del t, a
