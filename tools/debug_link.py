import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mini-kvstore-v2_amd"), os.path.join(ROOT, "tests")]
os.environ["KVR_DEBUG"] = "1"
import kvreplay as K, oracle_py as O
import test_gpu_parity as T
ctx = K.Context(0)
seg = T.boundary_segment()
for tps in (1,):
    ctx.set_tiles_per_stripe(tps)
    t0 = time.time()
    try:
        r = ctx.replay([seg])
        print("boundary tps", tps, "status", r.status, "redo rounds", r.stats.n_redo, "t", time.time() - t0, flush=True)
    except Exception as e:
        print("boundary tps", tps, "EXC", e, flush=True)
spec = K.GenSpec(seed=0x6B767265706C6179 + 2, seg_bytes=64 << 20, val_min=1024, val_max=1024, key_space_log2=20)
segs = [K.gen_segment_cpu(spec, s)[0] for s in range(8)]
for tps in (0,):
    ctx.set_tiles_per_stripe(tps)
    t0 = time.time()
    r = ctx.replay(segs)
    print("cfg2x4 tps", tps, "status", r.status, "redo rounds", r.stats.n_redo, "t", time.time() - t0, "ms_total", r.stats.ms_total, flush=True)
