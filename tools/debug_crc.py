"""Debug: device-generated cfg2 segments, replay with the manifest, compare failures with the oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mini-kvstore-v2_amd"), os.path.join(ROOT, "tests")]
import torch
import kvreplay as K, oracle_py as O

nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
seg_bytes = int(sys.argv[2]) if len(sys.argv) > 2 else (64 << 20)
spec = K.GenSpec(seed=0x6B767265706C6179 + 2, seg_bytes=seg_bytes, val_min=1024, val_max=1024, key_space_log2=20)
ctx = K.Context(0)
sizes = [K.gen_segment_size(spec, s) for s in range(nseg)]
offs, tot = [], 0
for ln, _ in sizes:
    offs.append(tot); tot += (ln + 255) & ~255
nrec = sum(n for _, n in sizes)
data = torch.empty(tot + 256, dtype=torch.uint8, device="cuda")
man = torch.empty(nrec + 1, dtype=torch.int32, device="cuda")
eo = 0
for s, (ln, nr), o in zip(range(nseg), sizes, offs):
    ctx.gen_segment_device(spec, s, data.data_ptr() + o, ln, man.data_ptr() + 4 * eo, nr); eo += nr
torch.cuda.synchronize()
segs = [(data.data_ptr() + o, ln) for (ln, _), o in zip(sizes, offs)]
for tps in (0, 1, 64):
    ctx.set_tiles_per_stripe(tps)
    r = ctx.replay(segs, on_device=True, expected=(man.data_ptr(), nrec), expected_on_device=True)
    t = r.tuples
    fails = np.nonzero(t["flags"] & K.TF_CRC_FAIL)[0]
    print(f"tps={tps} status={r.status} n={r.n}/{nrec} crc_fail={r.stats.n_crc_fail} stripes={r.stats.n_stripes}")
    if len(fails):
        host = [K.gen_segment_cpu(spec, s)[0] for s in range(nseg)]
        rc, ot, _ = O.replay(host)
        print("  oracle rc", rc, "n", len(ot), "eq", np.array_equal(ot["rec_off"], t["rec_off"]))
        exp = man[:nrec].cpu().numpy().view(np.uint32)
        for i in fails[:10]:
            print(f"  rec {i} seg {t['seg_idx'][i]} off {t['rec_off'][i]} tile {(t['rec_off'][i]) // 16384} "
                  f"gpu {t['crc32'][i]:08x} exp {exp[i]:08x} oracle {ot['crc32'][i]:08x}")
        d = np.nonzero(ot["crc32"] != t["crc32"])[0]
        print("  oracle-vs-gpu crc mismatches:", len(d), d[:10])
