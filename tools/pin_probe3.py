"""Registration granularity and file-backed memory on the GPU box (4 GiB):
  A  16 x 256 MiB hipHostRegister, sequential, on pre-faulted anonymous memory (vs 1 x 4 GiB)
  B  the same while 16 threads fault a second array (contention with page faults)
  C  files mmap'd (MAP_PRIVATE, populated): hipHostRegister rc + time, H2D registered / pageable"""
import ctypes as C
import mmap
import os
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
G = 1 << 30
TOT = 4 * G
P = 16
step = TOT // P
d = torch.empty(TOT, dtype=torch.uint8, device="cuda")


def faulted():
    a = np.empty(TOT, dtype=np.uint8)
    with ThreadPoolExecutor(P) as ex:
        list(ex.map(lambda i: a[i * step:(i + 1) * step].fill(1), range(P)))
    return a


for rnd in range(2):
    a = faulted()
    t0 = time.perf_counter()
    rcs = [hip.hipHostRegister(a.ctypes.data + i * step, step, 0) for i in range(P)]
    seq = time.perf_counter() - t0
    for i in range(P):
        hip.hipHostUnregister(a.ctypes.data + i * step)
    del a
    a = faulted()
    t0 = time.perf_counter()
    rc1 = hip.hipHostRegister(a.ctypes.data, TOT, 0)
    one = time.perf_counter() - t0
    hip.hipHostUnregister(a.ctypes.data)
    del a
    a = faulted()
    b = np.empty(TOT, dtype=np.uint8)
    with ThreadPoolExecutor(P + 1) as ex:
        fut = [ex.submit(lambda i=i: b[i * step:(i + 1) * step].fill(2)) for i in range(P)]
        t0 = time.perf_counter()
        rcs2 = [hip.hipHostRegister(a.ctypes.data + i * step, step, 0) for i in range(P)]
        con = time.perf_counter() - t0
        for f in fut:
            f.result()
    for i in range(P):
        hip.hipHostUnregister(a.ctypes.data + i * step)
    del a, b
    print(f"round {rnd}: 16x256MiB sequential {seq*1e3:.1f} ms {set(rcs)} | 1x4GiB {one*1e3:.1f} ms rc={rc1} | "
          f"16x256MiB during faults {con*1e3:.1f} ms {set(rcs2)}", flush=True)

tmpd = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
fn = os.path.join(tmpd, "seg.dat")
a = faulted()
with open(fn, "wb") as f:
    f.write(memoryview(a))
del a
for rnd in range(2):
    fd = os.open(fn, os.O_RDONLY)
    t0 = time.perf_counter()
    m = mmap.mmap(fd, TOT, flags=mmap.MAP_PRIVATE | getattr(mmap, "MAP_POPULATE", 0), prot=mmap.PROT_READ)
    mp = time.perf_counter() - t0
    arr = np.frombuffer(m, dtype=np.uint8)
    ptr = arr.ctypes.data
    t0 = time.perf_counter()
    h = torch.from_numpy(arr)   # read-only warning is harmless here
    d.copy_(h)
    torch.cuda.synchronize()
    pg = time.perf_counter() - t0
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ptr, TOT, 0)
    reg = time.perf_counter() - t0
    rg = float("nan")
    if rc == 0:
        t0 = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        rg = time.perf_counter() - t0
        hip.hipHostUnregister(ptr)
    del h, arr
    m.close()
    os.close(fd)
    print(f"round {rnd}: file mmap populate {mp*1e3:.1f} ms | H2D pageable mmap {pg*1e3:.1f} ms | register rc={rc} "
          f"{reg*1e3:.1f} ms | H2D registered {rg*1e3:.1f} ms", flush=True)
os.unlink(fn)
os.rmdir(tmpd)
