import sys, time, os
sys.path.insert(0, 'mini-kvstore-v2_amd'); sys.path.insert(0, '.')
import torch, ctypes as C, numpy as np
import kvreplay as K
ctx = K.Context(0)
spec = K.GenSpec(seed=1, seg_bytes=1 << 16, val_min=1024, val_max=1024, key_space_log2=20)
ln, nr = K.gen_segment_size(spec, 0)
data = torch.empty(ln + 256, dtype=torch.uint8, device='cuda')
man = torch.empty(nr + 1, dtype=torch.int32, device='cuda')
ctx.gen_segment_device(spec, 0, data.data_ptr(), ln, man.data_ptr(), nr)
torch.cuda.synchronize()
out = torch.empty((nr + 1024) * 32, dtype=torch.uint8, device='cuda')
sl = K.SegmentList([(data.data_ptr(), ln)], on_device=True)
def step():
    return ctx.replay(sl, expected=(man.data_ptr(), nr), expected_on_device=True, out_ptr=out.data_ptr(), cap=nr + 1024)
for _ in range(50): step()
t = time.perf_counter()
for _ in range(500): r = step()
dt = (time.perf_counter() - t) / 500 * 1e6
print(f"python step on a 64-KiB segment: {dt:.1f} us per call; ms_total {r.stats.ms_total*1000:.1f} us")
# raw ctypes
lib = ctx._lib if hasattr(ctx, '_lib') else None
print('attrs', [a for a in dir(ctx) if not a.startswith('__')][:30])
