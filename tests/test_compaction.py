"""Compaction live-record rewrite: oracle and GPU parity.

The reference's compaction (compaction.rs:9-29) deletes every segment and rewrites nothing
(SURVEY R3); its tests only check the in-process map (tests/store_integration.rs:20-32,
examples/compaction.rs:39-55).  The intended behaviour (README.md:283-287) is pinned instead:
  - a reference-semantics replay of the new segments gives the pre-compaction map (the same
    asserts, now across a reopen),
  - the output is exactly each key's final SET record, byte for byte, in (segment, offset)
    order (an independent Python restatement below),
  - a new segment starts at the first record at or after every multiple of seg_target.
GPU tests (marked gpu) compare kvr_compact with oracle_compact bit-exact through the C ABI.
"""
import os
import random
import shutil

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def rec_set(k, v):
    return b"\x00" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v


def rec_del(k):
    return b"\x01" + len(k).to_bytes(4, "little") + k


def read_dir(name):
    d = os.path.join(GOLD, name)
    names = sorted((n for n in os.listdir(d) if n.startswith("segment-")), key=lambda n: int(n[8:-4]))
    return [int(n[8:-4]) for n in names], [open(os.path.join(d, n), "rb").read() for n in names]


def walk(seg):
    """engine.rs:85-149 over one well-formed segment: (op, key, value, rec_off, rec_bytes)."""
    o, out = 0, []
    while o < len(seg):
        op = seg[o]
        kl = int.from_bytes(seg[o + 1: o + 5], "little")
        k = bytes(seg[o + 5: o + 5 + kl])
        if op == 0:
            vl = int.from_bytes(seg[o + 5 + kl: o + 9 + kl], "little")
            v = bytes(seg[o + 9 + kl: o + 9 + kl + vl])
            out.append((0, k, v, o, bytes(seg[o: o + 9 + kl + vl])))
            o += 9 + kl + vl
        else:
            out.append((1, k, None, o, None))
            o += 5 + kl
    return out


def py_map(segs):
    m = {}
    for s in segs:
        for op, k, v, _, _ in walk(s):
            if op == 0:
                m[k] = v
            else:
                m.pop(k, None)
    return m


def py_compact(segs, target):
    """Independent restatement: the final SET of every key, in (segment, offset) order."""
    recs = [r for s in segs for r in walk(s)]
    last = {}
    for i, (op, k, _, _, _) in enumerate(recs):
        last[k] = i
    out, ends, pos, nxt = bytearray(), [], 0, target
    for i, (op, k, _, _, rb) in enumerate(recs):
        if op != 0 or last[k] != i:
            continue
        if target and pos >= nxt:
            ends.append(pos)
            while nxt <= pos:
                nxt += target
        out += rb
        pos += len(rb)
    if pos:
        ends.append(pos)
    return bytes(out), ends


def gen_store(seed, n_segs=3, n_keys=200, n_recs=1500, dels=0.3, vmax=300):
    rng = random.Random(seed)
    segs = []
    for _ in range(n_segs):
        b = bytearray()
        for _ in range(n_recs // n_segs):
            k = f"key_{rng.randrange(n_keys)}".encode()
            if rng.random() < dels:
                b += rec_del(k)
            else:
                b += rec_set(k, bytes(rng.getrandbits(8) for _ in range(rng.randrange(vmax))))
        segs.append(bytes(b))
    return segs


# ---- the oracle, pinned ---------------------------------------------------------------------
@pytest.mark.parametrize("name,rounds", [("store_integration", 4), ("compaction_example", 9)])
def test_oracle_compact_reference_asserts(name, rounds):
    ids, segs = read_dir(name)
    rc, data, ends, _ = O.compact(segs, 0, seg_ids=ids)
    assert rc == 0 and len(ends) == 1 and ends[0] == len(data)
    new = O.split_segments(data, ends)
    m = py_map(new)   # a reopen of the new files
    # tests/store_integration.rs:22-31 / examples/compaction.rs:54-63, now across the reopen
    assert len(m) == 100
    for i in range(100):
        assert m[f"key_{i}".encode()] == f"value_{i}_{rounds}".encode()
    assert m == py_map(segs)
    assert (data, ends) == py_compact(segs, 0)


def test_oracle_compact_persistence_and_large():
    for name in ("persistence", "large_dataset"):
        ids, segs = read_dir(name)
        rc, data, ends, _ = O.compact(segs, 0, seg_ids=ids)
        assert rc == 0
        assert py_map(O.split_segments(data, ends)) == py_map(segs)
        assert (data, ends) == py_compact(segs, 0)


@pytest.mark.parametrize("target", [0, 1, 64, 1000, 4096, 1 << 40])
def test_oracle_compact_cut_rule(target):
    segs = gen_store(5, vmax=700)
    rc, data, ends, _ = O.compact(segs, target)
    assert rc == 0
    assert (data, ends) == py_compact(segs, target)
    new = O.split_segments(data, ends)
    assert py_map(new) == py_map(segs)
    assert all(len(s) > 0 for s in new)
    if target:   # every segment but the last starts below the next multiple: < target + one record
        starts = [0] + ends[:-1]
        for s, e in zip(starts, ends):
            nxt = (s // target + 1) * target
            last_start = max(o for _, _, _, o, _ in walk(data[s:e])) + s
            assert last_start < nxt


def test_oracle_compact_edge_cases():
    assert O.compact([], 0)[0] == 0
    rc, data, ends, _ = O.compact([rec_set(b"a", b"1") + rec_del(b"a")], 0)   # all deleted
    assert rc == 0 and data == b"" and ends == []
    rc, data, ends, _ = O.compact([b"", rec_set(b"a", b"")], 0)               # empty value, empty segment
    assert rc == 0 and data == rec_set(b"a", b"") and ends == [len(data)]
    bad = rec_set(b"a", b"1") + b"\x07" + (1).to_bytes(4, "little") + b"x"     # unknown opcode
    rc, _, _, err = O.compact([bad], 0)
    rc2, _, err2 = O.replay([bad])
    assert rc == rc2 == 1 and (err.kind, err.rec_off, err.aux) == (err2.kind, err2.rec_off, err2.aux)


# ---- the HIP path against the oracle ------------------------------------------------------------
def check_compact(ctx, segs, target, seg_ids=None):
    ro = O.compact(segs, target, seg_ids=seg_ids)
    rg = ctx.compact(segs, target, seg_ids=seg_ids)
    assert rg.status == ro[0]
    if ro[0] == 0:
        assert rg.seg_ends == ro[2]
        assert rg.data == ro[1]
    else:
        eo, eg = ro[3], rg.error
        assert (eg.kind, eg.seg_idx, eg.rec_off, eg.aux) == (eo.kind, eo.seg_idx, eo.rec_off, eo.aux)
    return rg


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["persistence", "store_integration", "compaction_example", "large_dataset"])
def test_gpu_compact_golden(gctx, name):
    ids, segs = read_dir(name)
    for target in (0, 100, 4096):
        check_compact(gctx, segs, target, seg_ids=ids)


SPECS = {
    "cfg4_del": K.GenSpec(seed=41, seg_bytes=600_000, val_min=1024, val_max=1024, del_permille=500,
                          key_space_log2=10),
    "cfg5_zipf": K.GenSpec(seed=51, seg_bytes=3_000_000, key_dist=1, key_space_log2=12, val_min=16,
                           val_max=1 << 18, del_permille=100),
    "tiny": K.GenSpec(seed=61, seg_bytes=200_000, val_min=0, val_max=40, del_permille=300, key_space_log2=8),
    "uniq": K.GenSpec(seed=62, seg_bytes=300_000, val_min=1, val_max=3000, key_space_log2=30),
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SPECS))
@pytest.mark.parametrize("target", [0, 1, 777, 65536])
def test_gpu_compact_generated(gctx, name, target):
    segs = [K.gen_segment_cpu(SPECS[name], s)[0] for s in range(3)]
    rg = check_compact(gctx, segs, target)
    assert rg.stats.n_tuples == len(O.replay(segs)[1])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SPECS))
def test_gpu_compact_two_scans(gctx, monkeypatch, name):
    """The rewrite's offsets and live positions from two scans over every tuple
    (KVR_COMPACT_TWO_SCANS) equal the byte-flag dense list's (k_dl_*) and the oracle's."""
    segs = [K.gen_segment_cpu(SPECS[name], s)[0] for s in range(3)]
    monkeypatch.setenv("KVR_COMPACT_TWO_SCANS", "1")
    check_compact(gctx, segs, 777)


@pytest.mark.gpu
def test_gpu_compact_python_stores(gctx):
    for seed in range(4):
        segs = gen_store(seed, n_keys=50 + 100 * seed, vmax=50 + 400 * seed)
        for target in (0, 1, 500):
            rg = check_compact(gctx, segs, target)
            assert (rg.data, rg.seg_ends) == py_compact(segs, target)


@pytest.mark.gpu
def test_gpu_compact_edges(gctx):
    check_compact(gctx, [rec_set(b"a", b"1") + rec_del(b"a")], 0)          # nothing live
    check_compact(gctx, [b"", rec_set(b"a", b""), b""], 0)                  # empty value / segments
    check_compact(gctx, [rec_set(b"k", b"v" * 100_000)] * 2, 10)            # one record over many multiples
    check_compact(gctx, [rec_set(b"a", b"1") + b"\x07\x01\x00\x00\x00x"], 0)   # corrupted: the replay error
    keys = [f"{i:03d}".encode() for i in range(300)]                        # 1-B values: 13-B records
    check_compact(gctx, [b"".join(rec_set(k, b"z") for k in keys)], 0)
    # the reported sizes
    segs = gen_store(9)
    ro = O.compact(segs, 100)
    r = gctx.compact(segs, 100)
    assert r.status == 0 and r.out_len == len(ro[1]) and r.n_segs == len(ro[2])


@pytest.mark.gpu
def test_gpu_compact_device_resident(gctx):
    torch = pytest.importorskip("torch")
    segs = [K.gen_segment_cpu(SPECS["cfg5_zipf"], s)[0] for s in range(3)]
    rc, data, ends, _ = O.compact(segs, 100_000)
    buf = torch.zeros(sum(len(s) for s in segs) + 4096, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 5
    for s in segs:
        buf[off: off + len(s)] = torch.from_numpy(s).cuda()
        ptrs.append((buf.data_ptr() + off, len(s)))
        off += len(s) + 3
    torch.cuda.synchronize()
    for shift in (0, 3):   # 8-B aligned output (direct) and an odd one (staged)
        out = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
        r = gctx.compact(ptrs, 100_000, on_device=True, out_ptr=out.data_ptr() + shift, out_cap=len(data) + 32)
        torch.cuda.synchronize()
        assert r.status == 0 and r.seg_ends == ends
        assert out[shift: shift + len(data)].cpu().numpy().tobytes() == data
        assert int(out[:shift].sum()) == 0 and int(out[shift + len(data):].sum()) == 0   # nothing outside
    small = torch.zeros(16, dtype=torch.uint8, device="cuda")
    r = gctx.compact(ptrs, 100_000, on_device=True, out_ptr=small.data_ptr(), out_cap=16)
    assert r.status == K.CAPACITY and r.out_len == len(data)


@pytest.mark.gpu
def test_gpu_compact_replay_property_large(gctx):
    """Size-independent property at a larger size: the compacted store's replay is exactly the
    live tuples of the original (keys, lengths, CRCs, in order)."""
    spec = K.GenSpec(seed=77, seg_bytes=8_000_000, val_min=1024, val_max=1024, del_permille=500,
                     key_space_log2=14)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(8)]
    r = gctx.compact(segs, 4 << 20)
    assert r.status == 0
    ro = gctx.replay(segs)
    live, nk, tb = O.fold_live(segs, ro.tuples)
    rn = gctx.replay(r.segments())
    assert rn.status == 0 and rn.n == nk == r.stats.n_live
    lt = ro.tuples[live]
    for f in ("key_len", "val_len", "crc32", "key_tag", "op"):
        assert np.array_equal(rn.tuples[f], lt[f]), f
    assert int(rn.tuples["val_len"].sum()) == tb


@pytest.mark.gpu
def test_kvstore_compact_then_reopen(gctx, tmp_path):
    """tests/store_integration.rs:12-31 and examples/compaction.rs, with the reopen the
    reference never does (its compact loses every key across a restart)."""
    for name, rounds in (("store_integration", 4), ("compaction_example", 9)):
        d = tmp_path / name
        shutil.copytree(os.path.join(GOLD, name), d)
        s = K.KVStore.open(str(d), gctx)
        before = s.stats()
        s.compact(seg_target=1000)
        for i in range(100):   # in-process asserts of the reference
            assert s.get(f"key_{i}") == f"value_{i}_{rounds}".encode()
        assert s.stats().num_keys == 100
        s.close()
        names = sorted(os.listdir(d))
        assert all(n.startswith("segment-") for n in names)
        s = K.KVStore.open(str(d), gctx)   # the reopen
        for i in range(100):
            assert s.get(f"key_{i}") == f"value_{i}_{rounds}".encode()
        st = s.stats()
        assert (st.num_keys, st.total_bytes) == (100, before.total_bytes)
        s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,target", [(2, 0), (3, 4096)])
def test_gpu_sharded_compaction(gctx, world, target):
    """The sharded compaction's device engine (kvr_compact_stage / _resolve / _finish) with the
    all-to-all exchanges emulated in-process (one context per rank on this one GPU): exports and
    answers equal the host engine's, and the ranks' outputs are exactly the global winners."""
    torch = pytest.importorskip("torch")
    from kvreplay import shard as SH
    from compact_cpu_engine import CAND, HostCompactEngine
    spec = K.GenSpec(seed=91, seg_bytes=400_000, val_min=1, val_max=2000, del_permille=400, key_space_log2=9)
    segs = [K.gen_segment_cpu(spec, s)[0].tobytes() for s in range(7)]
    ctxs = [gctx] + [K.Context(0) for _ in range(world - 1)]
    dev = [SH.DeviceCompactEngine(c, "cuda") for c in ctxs]
    host = [HostCompactEngine() for _ in range(world)]
    st_d, st_h = [], []
    for r in range(world):
        idx = SH.shard_round_robin(len(segs), world, r)
        st_d.append(dev[r].stage([segs[i] for i in idx], idx, world))
        st_h.append(host[r].stage([segs[i] for i in idx], idx, world))
        cd, kd, hd, ksd = st_d[r]
        ch, kh, hh, ksh = st_h[r]
        assert np.array_equal(cd, ch) and np.array_equal(kd, kh)
        assert hd.cpu().numpy().tobytes() == hh.numpy().tobytes()   # kvr_cand headers, in owner order
        hv, kbd, kbh = hh.numpy().view(CAND), ksd.cpu().numpy(), ksh.numpy()
        gk = np.concatenate([[0], np.cumsum(kh)])
        gh = np.concatenate([[0], np.cumsum(ch)])
        for o in range(world):                                       # key bytes (padding aside)
            for c in hv[gh[o]: gh[o + 1]]:
                a = gk[o] + c["key_off"]
                assert kbd[a: a + c["key_len"]].tobytes() == kbh[a: a + c["key_len"]].tobytes()

    def group(r, o):   # rank r's headers / keys for owner o
        c, kb, h, k = st_d[r]
        hs, ks = np.concatenate([[0], np.cumsum(c)]), np.concatenate([[0], np.cumsum(kb)])
        return h[hs[o] * 24: hs[o + 1] * 24], k[ks[o]: ks[o + 1]], int(c[o]), int(kb[o])

    wins = []
    for o in range(world):                                           # owners resolve
        parts = [group(s, o) for s in range(world)]
        hdr_in = torch.cat([p[0] for p in parts])
        keys_in = torch.cat([p[1] for p in parts])
        rc_counts = np.array([p[2] for p in parts], dtype=np.int64)
        rc_keys = np.array([p[3] for p in parts], dtype=np.int64)
        w = dev[o].resolve(hdr_in, keys_in, rc_counts, rc_keys)
        wh = host[o].resolve(hdr_in.cpu(), keys_in.cpu(), rc_counts, rc_keys)
        assert np.array_equal(w.cpu().numpy(), wh.numpy())
        wins.append((w, np.concatenate([[0], np.cumsum(rc_counts)])))
    outs = []
    for r in range(world):                                           # answers back, finish
        win_mine = torch.cat([wins[o][0][wins[o][1][r]: wins[o][1][r + 1]] for o in range(world)])
        outs.append(dev[r].finish(win_mine, target))
    # expected: the global last record of every key that is a SET, on the rank holding it
    rc, t, _ = O.replay(segs)
    last = {}
    for i, rr in enumerate(t):
        s = segs[rr["seg_idx"]]
        last[s[rr["rec_off"] + 5: rr["rec_off"] + 5 + rr["key_len"]]] = i
    exp = [bytearray() for _ in range(world)]
    for i in sorted(last.values()):
        rr = t[i]
        if rr["op"] == 0:
            s = segs[rr["seg_idx"]]
            exp[rr["seg_idx"] % world] += s[rr["rec_off"]: rr["rec_off"] + 9 + rr["key_len"] + rr["val_len"]]
    for r in range(world):
        assert outs[r][0] == bytes(exp[r])
        assert py_compact([outs[r][0]], target)[1] == outs[r][1]     # the cut rule on each rank's output
    for c in ctxs[1:]:
        c.close()
