"""Timing tool: the fold on a skewed store (log-uniform keys, kvr_gen_common.h key_dist 1: key 0
alone takes 1/20 of the records) at cfg4's shape, through kvr_compact and kvr_replay_live.
Prints the per-phase times of a few calls; run it with and without KVR_FOLD_GLOBAL=1.
    python tools/fold_skew.py [segments] [calls]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-kvstore-v2_amd"))
import kvreplay as K  # noqa: E402


def main():
    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    spec = K.GenSpec(seed=0x5EED4, seg_bytes=64 << 20, key_space_log2=20, key_dist=1, val_min=1024,
                     val_max=1024, del_permille=500)
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
    segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
    out = torch.empty(tot + 4096, dtype=torch.uint8, device="cuda")
    mode = "global" if os.environ.get("KVR_FOLD_GLOBAL") else "partitioned"
    for i in range(calls):
        t0 = time.perf_counter()
        r = ctx.compact(segs, 64 << 20, on_device=True, out_ptr=out.data_ptr(), out_cap=out.numel())
        ms = (time.perf_counter() - t0) * 1e3
        assert r.status == 0
        print(f"{mode} compact {i}: wall {ms:.3f} ms  replay {r.stats.ms_replay:.3f}  fold {r.stats.ms_fold:.3f}  "
              f"gather {r.stats.ms_gather:.3f}  tuples {r.stats.n_tuples}  live {r.stats.n_live}", flush=True)
    for i in range(calls):
        t0 = time.perf_counter()
        lv = ctx.replay_live(segs, on_device=True)
        ms = (time.perf_counter() - t0) * 1e3
        assert lv.status == 0
        print(f"{mode} replay_live {i}: wall {ms:.3f} ms  live {len(lv.tuples)}", flush=True)


if __name__ == "__main__":
    main()
