"""Device index on the cfg2 shard, device-resident (for rocprofv3 --kernel-trace --stats):
kvr_replay_index x N with segments in HBM; prints the index stats per call."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mini-kvstore-v2_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import kvreplay as K
from bench import CONFIGS

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nseg, seg_bytes, kw, desc = CONFIGS[cfg]
spec = K.GenSpec(seed=0x6B767265706C6179 + int(cfg[3:]), seg_bytes=seg_bytes, **kw)
ctx = K.Context(0)
sizes = [K.gen_segment_size(spec, s) for s in range(nseg)]
offs, tot = [], 0
for ln, _ in sizes:
    offs.append(tot)
    tot += (ln + 255) & ~255
data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda")
n_rec = sum(nr for _, nr in sizes)
man = torch.empty(n_rec + 1, dtype=torch.int32, device="cuda")
eo = 0
for s, (ln, nr), o in zip(range(nseg), sizes, offs):
    ctx.gen_segment_device(spec, s, data.data_ptr() + o, ln, man.data_ptr() + 4 * eo, nr)
    eo += nr
torch.cuda.synchronize()
segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
if len(sys.argv) > 3 and sys.argv[3] == "plain":   # plain replays first (no key prefixes): k_piece with and without
    out = torch.empty((n_rec + 1024) * 32, dtype=torch.uint8, device="cuda")
    for i in range(reps):
        r = ctx.replay(segs, on_device=True, out_ptr=out.data_ptr(), cap=n_rec + 1024)
        print(f"{cfg} plain replay: ms_replay {r.stats.ms_replay:.3f} ms_total {r.stats.ms_total:.3f}", flush=True)
for i in range(reps):
    ix = ctx.replay_index(segs, on_device=True)
    st = ix.stats
    print(f"{cfg} replay_index: wall {st.ms_wall:.3f} ms  replay {st.ms_replay:.3f}  fold+live+table {st.ms_fold:.3f}  "
          f"tuples {st.n_tuples} live {st.n_live} rounds {st.fold_rounds} est {st.fold_est} slots {st.fold_slots} "
          f"redo {st.fold_redo}", flush=True)
