"""Host restatement of the sharded-compaction engine (stage / resolve / finish).

TEST INFRASTRUCTURE: it stands in for kvreplay.shard.DeviceCompactEngine (the HIP kernels of
kvr_compact_stage / _resolve / _finish) in the world_size-2 gloo tests that run without a GPU, and
it is the checker the GPU test compares the device engine's exports and answers with.  Built on
the CPU oracle's replay (oracle/replay_ref.c); the wire format is the C ABI's kvr_cand.
"""
import numpy as np
import torch

import oracle_py as O

CAND = np.dtype([("pos", "<u8"), ("key_len", "<u4"), ("key_tag", "<u4"), ("key_off", "<u4"), ("pad", "<u4")])
M32 = 0xFFFFFFFF


def ht_mix(h):
    h ^= h >> 16
    h = (h * 0x7FEB352D) & M32
    h ^= h >> 15
    h = (h * 0x846CA68B) & M32
    h ^= h >> 16
    return h


def owner_of(tag, world):
    return (ht_mix(int(tag)) >> 7) % world


class HostCompactEngine:
    def stage(self, segments, gidx, world, on_device=False):
        self.segs = [bytes(s) for s in segments]
        rc, t, err = O.replay(self.segs)
        if rc != 0:
            raise RuntimeError(f"replay failed {rc}")
        self.t = t
        last = {}
        for i, r in enumerate(t):
            last[self._key(r)] = i
        self.cand = sorted(last.values())                     # tuple order
        groups = [[i for i in self.cand if owner_of(t[i]["key_tag"], world) == o] for o in range(world)]
        self.export_order = [i for g in groups for i in g]
        hdr, keys, counts, kb = [], bytearray(), [], []
        for g in groups:
            koff = 0
            for i in g:
                r = t[i]
                k = self._key(r)
                hdr.append((int(gidx[r["seg_idx"]]) << 40 | int(r["rec_off"]), len(k), int(r["key_tag"]), koff, 0))
                pad = (len(k) + 3) & ~3
                keys += k + b"\0" * (pad - len(k))
                koff += pad
            counts.append(len(g))
            kb.append(koff)
        h = np.array(hdr, dtype=CAND)
        return (np.array(counts, dtype=np.int64), np.array(kb, dtype=np.int64),
                torch.from_numpy(h.view(np.uint8).copy()), torch.frombuffer(bytearray(keys), dtype=torch.uint8)
                if keys else torch.empty(0, dtype=torch.uint8))

    def resolve(self, hdr, keys, hdr_counts, key_counts):
        h = hdr.numpy().view(CAND) if hdr.numel() else np.zeros(0, CAND)
        kbytes = keys.numpy().tobytes()
        hs = np.concatenate([[0], np.cumsum(hdr_counts)])
        ks = np.concatenate([[0], np.cumsum(key_counts)])
        best, names = {}, []
        for i, c in enumerate(h):
            s = int(np.searchsorted(hs, i, side="right") - 1)
            k = kbytes[ks[s] + c["key_off"]: ks[s] + c["key_off"] + c["key_len"]]
            names.append(k)
            best[k] = max(best.get(k, 0), int(c["pos"]))
        win = [1 if int(c["pos"]) == best[k] else 0 for c, k in zip(h, names)]
        return torch.tensor(win, dtype=torch.uint8)

    def finish(self, win, seg_target):
        w = dict(zip(self.export_order, win.numpy().tolist()))
        out, ends, pos, nxt = bytearray(), [], 0, seg_target
        for i in self.cand:
            r = self.t[i]
            if r["op"] != 0 or not w[i]:
                continue
            if seg_target and pos >= nxt:
                ends.append(pos)
                while nxt <= pos:
                    nxt += seg_target
            sz = 9 + int(r["key_len"]) + int(r["val_len"])
            out += self.segs[r["seg_idx"]][r["rec_off"]: r["rec_off"] + sz]
            pos += sz
        if pos:
            ends.append(pos)
        return bytes(out), ends

    def _key(self, r):
        s = self.segs[r["seg_idx"]]
        return s[r["rec_off"] + 5: r["rec_off"] + 5 + r["key_len"]]
