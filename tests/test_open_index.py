"""The open-time index (kvr_replay_index / kvr_ingest_*, kvs_open_ex) and the fold's tag rounds.

Parity: the live list is exactly the oracle's (oracle_fold_live: engine.rs:137 insert / :141
remove over oracle_replay's tuples, in (segment, offset) order), every live key is found at its
live index through the table, and every other key is absent (engine.rs:200 get -> None).

The fold compares key bytes only when the CRC-32 tags match; keys that share a CRC-32 are found
here by brute force (zlib.crc32 over a fixed key set, deterministic), so the collision rounds of
k_fold_verify run on real collisions: same-length short keys, and long keys whose first 16 bytes
(the part the fold entry holds) are equal too.
"""
import os
import shutil
import zlib

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rec_set(k, v):
    return b"\x00" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v


def rec_del(k):
    return b"\x01" + len(k).to_bytes(4, "little") + k


def crc_collisions(prefix, n, want):
    """Pairs of distinct keys prefix + 16 hex digits of a scrambled i (i < n) with equal CRC-32, up
    to want pairs.  (Keys differing only in a few trailing bytes never collide: CRC-32 catches
    every burst of up to 32 bits, so the varying part is spread over 16 bytes.)"""
    seen, pairs = {}, []
    for i in range(n):
        k = prefix + b"%016x" % ((i * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
        c = zlib.crc32(k)
        if c in seen:
            pairs.append((seen[c], k))
            if len(pairs) >= want:
                break
        else:
            seen[c] = k
    return pairs


def collision_store():
    """Segments whose keys include CRC-32-colliding pairs, with SETs, overwrites and DELs."""
    short = crc_collisions(b"", 400_000, 6)
    long_ = crc_collisions(b"shared-prefix-16-tail-", 400_000, 6)
    pairs = short + long_
    assert len(short) >= 3 and len(long_) >= 3
    assert all(len(a) == len(b) and a != b and zlib.crc32(a) == zlib.crc32(b) for a, b in pairs)
    assert all(a[:16] == b[:16] for a, b in long_)
    segs = []
    for s in range(4):
        b = bytearray()
        for j, (a, c) in enumerate(pairs):
            # per pair and segment: a different mix of writes to the two keys
            m = (s * 7 + j) % 5
            if m == 0:
                b += rec_set(a, b"A%d-%d" % (s, j)) + rec_set(c, b"C%d-%d" % (s, j))
            elif m == 1:
                b += rec_set(c, b"c%d" % s) + rec_del(a)
            elif m == 2:
                b += rec_del(c) + rec_set(a, b"a%d" % s) + rec_set(a, b"aa%d" % s)
            elif m == 3:
                b += rec_set(a, b"") + rec_set(c, b"x" * (j + s))
            else:
                b += rec_del(a) + rec_del(c)
            b += rec_set(b"plain-%d-%d" % (s, j), b"v")
        segs.append(bytes(b))
    return segs, pairs


def expect(segs, seg_ids=None):
    rc, t, err = O.replay(segs, seg_ids=seg_ids)
    assert rc == 0
    live, nk, tb = O.fold_live(segs, t)
    return t[live], nk, tb


def keys_of(segs, tuples):
    return [bytes(segs[t["seg_idx"]][t["rec_off"] + 5: t["rec_off"] + 5 + t["key_len"]]) for t in tuples]


DEAD = 0xFFFFFFFF


def check_index(idx, segs, want, absent=()):
    assert np.array_equal(idx.live, want)
    ns = len(idx.slots)
    assert ns >= 16 and ns & (ns - 1) == 0 and ns > len(want)
    used = idx.slots[(idx.slots != 0) & (idx.slots != DEAD)]
    assert len(used) == len(want) and len(np.unique(used)) == len(want)
    for j, k in enumerate(keys_of(segs, want)):
        assert idx.find(k, segs) == j
    for k in absent:
        assert idx.find(k, segs) == -1


# ---- host side (no GPU): the table layout and the lookup ----------------------------------------
def test_index_build_host_and_find():
    segs, pairs = collision_store()
    want, nk, _ = expect(segs)
    slots = K.index_build_host(want)
    idx = K.Index(want, slots, segs, None)
    live_keys = set(keys_of(segs, want))
    absent = [k for p in pairs for k in p if k not in live_keys] + [b"never-written", b""]
    check_index(idx, segs, want, absent)
    # every entry sits on its probe path: home slot, then linear probing without a free slot between
    mask = len(slots) - 1
    for h in np.nonzero(slots)[0]:
        home = K.index_hash(int(want[slots[h] - 1]["key_tag"])) & mask
        p = home
        while p != h:
            assert slots[p] != 0
            p = (p + 1) & mask
    assert len(K.index_build_host(want[:0])) == 16


# ---- device index --------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("path", ["lds", "global"])
def test_fold_tag_collisions(gctx, monkeypatch, path):
    """Distinct keys with equal CRC-32 (short, and long with equal 16-B prefixes) fold exactly, in
    the partitioned fold's LDS ranges and in the global claim rounds (KVR_FOLD_GLOBAL)."""
    if path == "global":
        monkeypatch.setenv("KVR_FOLD_GLOBAL", "1")
    segs, pairs = collision_store()
    want, nk, tb = expect(segs)
    r = gctx.replay_live(segs)
    assert r.status == 0 and np.array_equal(r.tuples, want)
    idx = gctx.replay_index(segs)
    live_keys = set(keys_of(segs, want))
    check_index(idx, segs, want, [k for p in pairs for k in p if k not in live_keys])
    # the global claims take a collision to a further round; the LDS ranges resolve it in place
    assert idx.stats.fold_rounds >= (2 if path == "global" else 1) and idx.stats.n_live == nk
    # the rewrite uses the same fold: its output replays to the same map
    c = gctx.compact(segs)
    rc, t2, _ = O.replay(c.segments())
    assert rc == 0 and len(t2) == nk


@pytest.mark.gpu
def test_fold_table_redo(gctx, monkeypatch):
    """A fold table sized below the distinct keys (forced to 16 entries) fills up; the fold is
    redone at 2 n entries and gives the same answer."""
    segs, pairs = collision_store()
    want, nk, _ = expect(segs)
    monkeypatch.setenv("KVR_FOLD_TINY_TABLE", "1")
    idx = gctx.replay_index(segs)
    assert idx.stats.fold_redo == 1 and np.array_equal(idx.live, want)
    monkeypatch.delenv("KVR_FOLD_TINY_TABLE")
    idx = gctx.replay_index(segs)
    assert idx.stats.fold_redo == 0 and np.array_equal(idx.live, want)


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["prefixes", "segments", "batched"])
def test_fold_key_sources(gctx, monkeypatch, source):
    """The fold compares keys through the 16-B prefixes k_replay wrote beside the tuples (the
    default for calls that fold), or through the segment bytes (KVR_FOLD_SEGKEYS, and a replay
    batched past the pool-slot limit, which writes no prefixes): the same live index, CRC-32
    collisions and short keys included, and the rewrite built on it replays to the same map."""
    segs, pairs = collision_store()
    spec = K.GenSpec(seed=105, seg_bytes=200_000, key_space_log2=10, val_min=0, val_max=300, del_permille=300)
    segs = segs + [K.gen_segment_cpu(spec, s)[0].tobytes() for s in range(6)]
    want, nk, _ = expect(segs)
    if source == "segments":
        monkeypatch.setenv("KVR_FOLD_SEGKEYS", "1")
    if source == "batched":
        monkeypatch.setenv("KVR_POOL_LIMIT", "200000")
    r = gctx.replay_live(segs)
    assert r.status == 0 and np.array_equal(r.tuples, want)
    idx = gctx.replay_index(segs)
    assert np.array_equal(idx.live, want) and idx.stats.n_live == nk
    c = gctx.compact(segs)
    rc, t2, _ = O.replay(c.segments())
    assert rc == 0 and len(t2) == nk
    assert sorted(keys_of(c.segments(), t2)) == sorted(keys_of(segs, want))


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["global", "range16", "range64", "bucket32", "range16-bucket32"])
def test_fold_partition_overflow(gctx, monkeypatch, path):
    """The partitioned fold hands a tuple to the global rounds when its probe runs off the end of
    its LDS range (KVR_FOLD_RANGE: ranges of 16 / 64 entries) or it comes after the first 32
    records of its bucket (KVR_FOLD_BUCKET); those rounds go on probing in the table the ranges wrote.  Same
    live index (CRC-32 collisions included) and rewrite as the reference fold."""
    segs, pairs = collision_store()
    spec = K.GenSpec(seed=107, seg_bytes=150_000, key_space_log2=11, val_min=0, val_max=200, del_permille=250)
    segs = segs + [K.gen_segment_cpu(spec, s)[0].tobytes() for s in range(5)]
    want, nk, _ = expect(segs)
    if path == "global":
        monkeypatch.setenv("KVR_FOLD_GLOBAL", "1")
    if "range" in path:
        monkeypatch.setenv("KVR_FOLD_RANGE", path.split("-")[0][5:])
    if "bucket" in path:
        monkeypatch.setenv("KVR_FOLD_BUCKET", "32")
    r = gctx.replay_live(segs)
    assert r.status == 0 and np.array_equal(r.tuples, want)
    idx = gctx.replay_index(segs)
    live_keys = set(keys_of(segs, want))
    check_index(idx, segs, want, [k for p in pairs for k in p if k not in live_keys])
    assert idx.stats.n_live == nk
    if path != "global" and path != "range64":   # (64-entry ranges may hold every probe)
        assert idx.stats.fold_rounds >= 2   # some tuples went on to the global rounds
    c = gctx.compact(segs)
    rc, t2, _ = O.replay(c.segments())
    assert rc == 0 and len(t2) == nk
    assert sorted(keys_of(c.segments(), t2)) == sorted(keys_of(segs, want))


@pytest.mark.gpu
def test_fold_hot_keys(gctx, monkeypatch):
    """Log-uniform keys over 2^20 (kvr_gen_common.h key_dist 1: key 0 alone is 1/20 of the
    records, keys 1-2 1/40 each, ...) in 2 M small records: the hot keys' table ranges pass their
    LDS cap and leave their earlier records to k_fold_hot.  The live list, the key table and the
    rewrite equal the oracle's; the global claims (KVR_FOLD_GLOBAL) give the same live list and a
    key table as valid."""
    spec = K.GenSpec(seed=211, seg_bytes=8 << 20, key_space_log2=20, key_dist=1, val_min=0, val_max=16,
                     del_permille=300)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(8)]
    want, nk, _ = expect(segs)
    r = gctx.replay_live(segs)
    assert r.status == 0 and np.array_equal(r.tuples, want)
    idx = gctx.replay_index(segs)
    check_index(idx, segs, want, [b"no-such-key"])
    assert idx.stats.n_tuples > 2_000_000 and idx.stats.n_live == nk
    monkeypatch.setenv("KVR_FOLD_GLOBAL", "1")
    idx_g = gctx.replay_index(segs)
    check_index(idx_g, segs, want, [b"no-such-key"])   # (entries may sit elsewhere: another claim order)
    monkeypatch.delenv("KVR_FOLD_GLOBAL")
    c = gctx.compact(segs, 4 << 20)
    rc, want_c, ends, _ = O.compact(segs, 4 << 20)
    assert rc == 0 and c.status == 0 and c.seg_ends == ends and c.data == want_c


@pytest.mark.gpu
def test_fold_table_estimate(gctx):
    """cfg-like input with many more tuples than keys: the table is sized from the HyperLogLog
    estimate (within a few percent of the true key count), not from the tuples."""
    spec = K.GenSpec(seed=100, seg_bytes=8_000_000, key_space_log2=15, val_min=8, val_max=64, del_permille=0)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(4)]
    want, nk, _ = expect(segs)
    idx = gctx.replay_index(segs)
    st = idx.stats
    assert np.array_equal(idx.live, want) and st.n_tuples > 8 * nk
    assert abs(st.fold_est - nk) < 0.05 * nk
    assert st.fold_slots < st.n_tuples and st.fold_slots >= 1.6 * st.fold_est


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["persistence", "store_integration", "compaction_example", "large_dataset"])
def test_replay_index_golden(gctx, name):
    d = os.path.join(GOLD, name)
    names = sorted((n for n in os.listdir(d) if n.startswith("segment-")), key=lambda n: int(n[8:-4]))
    segs = [open(os.path.join(d, n), "rb").read() for n in names]
    ids = [int(n[8:-4]) for n in names]
    want, nk, _ = expect(segs, ids)
    idx = gctx.replay_index(segs, seg_ids=ids)
    check_index(idx, segs, want, [b"no-such-key"])
    for pinned in (False, True):
        ig = gctx.ingest_index(segs, seg_ids=ids, pinned=pinned)
        check_index(ig, segs, want)


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [
    K.GenSpec(seed=95, seg_bytes=600_000, key_space_log2=12, val_min=0, val_max=200, del_permille=300),
    K.GenSpec(seed=96, seg_bytes=3_000_000, key_dist=1, key_space_log2=20, val_min=8, val_max=4096,
              del_permille=50),
])
def test_replay_index_generated(gctx, spec):
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(6)]
    want, nk, tb = expect(segs)
    idx = gctx.replay_index(segs)
    assert np.array_equal(idx.live, want) and idx.stats.n_live == nk
    used = idx.slots[(idx.slots != 0) & (idx.slots != DEAD)]
    assert len(used) == nk and len(np.unique(used)) == nk
    ks = keys_of(segs, want)
    for j in range(0, nk, max(1, nk // 300)):
        assert idx.find(ks[j], segs) == j
    ig = gctx.ingest_index(segs, pinned=True)
    assert np.array_equal(ig.live, want)
    assert all(ig.find(ks[j], segs) == j for j in range(0, nk, max(1, nk // 100)))


@pytest.mark.gpu
def test_replay_index_errors(gctx):
    spec = K.GenSpec(seed=97, seg_bytes=200_000, key_space_log2=8, val_min=0, val_max=64, del_permille=300)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(3)]
    bad = segs[:1] + [segs[1][:-2]] + segs[2:]
    rc, _, err = O.replay(bad)
    r = gctx.replay_index(bad)
    assert r.status == rc == 1 and (r.error.kind, r.error.seg_idx, r.error.rec_off) == (err.kind, err.seg_idx, err.rec_off)
    r = gctx.ingest_index(bad)
    assert r.status == 1 and (r.error.kind, r.error.seg_idx, r.error.rec_off) == (err.kind, err.seg_idx, err.rec_off)
    e = gctx.replay_index([])
    assert len(e.live) == 0 and len(e.slots) == 16 and e.find(b"x", []) == -1


@pytest.mark.gpu
def test_live_index_device_buffers(gctx):
    """kvr_replay_live with segments in HBM (KVR_SEGS_ON_DEVICE) and tuples left in HBM
    (KVR_OUT_ON_DEVICE), and its KVR_CAPACITY answer for a device buffer."""
    torch = pytest.importorskip("torch")
    spec = K.GenSpec(seed=98, seg_bytes=500_000, key_space_log2=11, val_min=0, val_max=300, del_permille=250)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(4)]
    want, nk, _ = expect(segs)
    buf = torch.zeros(sum(len(s) + 64 for s in segs), dtype=torch.uint8, device="cuda")
    ptrs, off = [], 5
    for s in segs:
        buf[off: off + len(s)] = torch.from_numpy(s).cuda()
        ptrs.append((buf.data_ptr() + off, len(s)))
        off += len(s) + 9
    torch.cuda.synchronize()
    out = torch.zeros((nk + 8) * 32, dtype=torch.uint8, device="cuda")
    r = gctx.replay_live(ptrs, on_device=True, out_ptr=out.data_ptr(), cap=nk + 8)
    assert r.status == 0 and r.n == nk
    got = out[: nk * 32].cpu().numpy().view(K.TUPLE_DTYPE)
    assert np.array_equal(got, want)
    r = gctx.replay_live(ptrs, on_device=True, out_ptr=out.data_ptr(), cap=nk - 1)
    assert r.status == K.CAPACITY and r.n == nk
    r = gctx.replay_live(ptrs, on_device=True)   # segments in HBM, tuples to the host
    assert r.status == 0 and np.array_equal(r.tuples, want)


# ---- kvs_open_ex: the files -> index path ---------------------------------------------------------
def _write_store(d, segs, ids):
    d.mkdir()
    for i, s in zip(ids, segs):
        (d / f"segment-{i}.dat").write_bytes(bytes(s))


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, K.OPEN_NO_PIN, K.OPEN_PREAD, K.OPEN_PREAD | K.OPEN_NO_PIN, K.OPEN_HOST_FOLD,
                                   K.OPEN_HOST_FOLD | K.OPEN_PREAD])
def test_kvs_open_paths_agree(gctx, tmp_path, flags):
    spec = K.GenSpec(seed=99, seg_bytes=900_000, key_space_log2=12, val_min=0, val_max=500, del_permille=200)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(7)]
    segs[2] = segs[2][:0]   # an empty segment file (a fresh active segment) among them
    ids = [3, 4, 10, 11, 12, 40, 41]
    d = tmp_path / "db"
    _write_store(d, segs, ids)
    want, nk, tb = expect(segs, ids)
    s = K.KVStore.open(str(d), gctx, flags=flags)
    st = s.stats()
    assert (st.num_keys, st.total_bytes, st.active_segment_id) == (nk, tb, 42)
    os_ = s.open_stats()
    assert os_.path == (K.PATH_HOST_FOLD if flags & K.OPEN_HOST_FOLD else K.PATH_DEVICE_INDEX)
    assert os_.bytes == sum(len(x) for x in segs) and os_.n_segments == 7 and os_.n_live == nk
    assert os_.mode == (K.LOAD_PREAD if flags & K.OPEN_PREAD else K.LOAD_MMAP)
    for t, k in list(zip(want, keys_of(segs, want)))[:: max(1, nk // 200)]:
        vo = t["rec_off"] + 9 + t["key_len"]
        assert s.get(k) == bytes(segs[t["seg_idx"]][vo: vo + t["val_len"]])
        assert s.locate(k) == (ids[t["seg_idx"]], vo, t["val_len"])
    assert s.get(b"absent-key") is None
    s.compact(seg_target=1 << 20)   # the rebuild after compaction uses the store's path too
    assert s.stats().num_keys == nk and s.stats().total_bytes == tb
    k0 = keys_of(segs, want[:1])[0]
    v0 = want[0]
    assert s.get(k0) == bytes(segs[v0["seg_idx"]][v0["rec_off"] + 9 + v0["key_len"]:][: v0["val_len"]])
    s.close()


@pytest.mark.gpu
def test_kvs_open_unopenable_segment_order(gctx, tmp_path):
    """engine.rs:55-57 opens segment k after 0 .. k-1 replayed: an earlier corruption wins over a
    later unopenable file; with clean segments before it, the open error is reported."""
    d = tmp_path / "db"
    d.mkdir()
    (d / "segment-1.dat").write_bytes(rec_set(b"a", b"1"))
    os.symlink(str(d / "missing-target"), str(d / "segment-2.dat"))
    (d / "segment-3.dat").write_bytes(rec_set(b"b", b"2"))
    with pytest.raises(K.CorruptedData) as ei:
        K.KVStore.open(str(d), gctx)
    assert (ei.value.kind, ei.value.seg_idx) == (K.E_OPEN, 1)
    assert str(ei.value) == (f"Corrupted data: Failed to open segment {d}/segment-2.dat: "
                             f"No such file or directory (os error 2)")
    (d / "segment-1.dat").write_bytes(rec_set(b"a", b"1") + b"\x00\x05")
    with pytest.raises(K.CorruptedData) as ei:
        K.KVStore.open(str(d), gctx)
    assert (ei.value.kind, ei.value.seg_idx) == (K.E_KEY_LEN, 0)


@pytest.mark.gpu
def test_kvs_open_golden_host_fold(gctx, tmp_path):
    d = tmp_path / "persisted_store"
    shutil.copytree(os.path.join(GOLD, "persistence"), d)
    s = K.KVStore.open(str(d), gctx, flags=K.OPEN_HOST_FOLD)
    assert s.get("session") == b"first" and s.get("counter") == b"43" and s.get("name") is None
    assert s.locate("counter") == (2, 16, 2)
    assert (s.stats().num_keys, s.stats().total_bytes) == (2, 7)
    s.close()


@pytest.mark.gpu
def test_live_keys_arena(gctx):
    """kvr_live_keys: the live keys' bytes packed in live order equal the oracle's key bytes —
    from host segments (replay_index), from segments in HBM (replay_live on device pointers, the
    host holding no bytes) and after an ingest."""
    torch = pytest.importorskip("torch")
    segs, pairs = collision_store()
    spec = K.GenSpec(seed=101, seg_bytes=300_000, key_space_log2=10, val_min=0, val_max=100, del_permille=300)
    segs = segs + [K.gen_segment_cpu(spec, s)[0] for s in range(3)]
    want, nk, _ = expect(segs)
    wkeys = keys_of(segs, want)

    def check(n):
        keys, offs = gctx.live_keys(n)
        assert n == nk and offs[0] == 0 and int(offs[-1]) == len(keys) == sum(len(k) for k in wkeys)
        assert [bytes(keys[offs[i]: offs[i + 1]]) for i in range(n)] == wkeys

    idx = gctx.replay_index(segs)
    check(len(idx.live))
    buf = torch.zeros(sum(len(x) + 16 for x in segs), dtype=torch.uint8, device="cuda")
    ptrs, off = [], 1
    for x in segs:
        buf[off: off + len(x)] = torch.from_numpy(np.frombuffer(bytes(x), dtype=np.uint8).copy()).cuda()
        ptrs.append((buf.data_ptr() + off, len(x)))
        off += len(x) + 3
    torch.cuda.synchronize()
    r = gctx.replay_live(ptrs, on_device=True)
    assert r.status == 0 and np.array_equal(r.tuples, want)
    check(r.n)
    ig = gctx.ingest_index(segs, pinned=True)
    check(len(ig.live))
    gctx.replay_live([])
    k, o = gctx.live_keys(0)
    assert len(k) == 0 and list(o) == [0]


@pytest.mark.gpu
def test_replay_batches_past_pool_limit(gctx, monkeypatch):
    """A replay whose tuple pool would exceed the 32-bit slot limit runs as consecutive batches
    of whole segments (the limit lowered by KVR_POOL_LIMIT): same tuples, CRC verification, first
    error and device output as one pass."""
    torch = pytest.importorskip("torch")
    spec = K.GenSpec(seed=102, seg_bytes=300_000, key_space_log2=12, val_min=0, val_max=400, del_permille=200,
                     flip_per_million=3000)
    parts = [K.gen_segment_cpu(spec, s) for s in range(12)]
    segs = [p[0] for p in parts]
    man = np.concatenate([p[1] for p in parts])
    rc, want, _ = O.replay(segs, expected=man)
    assert rc == 0 and (want["flags"] & K.TF_CRC_FAIL).any()
    monkeypatch.setenv("KVR_POOL_LIMIT", "400000")
    r = gctx.replay(segs, expected=man)
    assert r.status == 0 and np.array_equal(r.tuples, want)
    assert r.stats.n_records == len(want) and r.stats.n_crc_fail == int((want["flags"] & K.TF_CRC_FAIL != 0).sum())
    bad = segs[:9] + [segs[9][:-3]] + segs[10:]
    rc, _, err = O.replay(bad)
    r = gctx.replay(bad)
    assert r.status == 1 and (r.error.kind, r.error.seg_idx, r.error.rec_off) == (err.kind, err.seg_idx, err.rec_off)
    out = torch.zeros((len(want) + 8) * 32, dtype=torch.uint8, device="cuda")
    r = gctx.replay(segs, on_device=False, out_ptr=out.data_ptr(), cap=len(want) + 8)
    assert r.status == 0 and r.n == len(want)
    got = out[: len(want) * 32].cpu().numpy().view(K.TUPLE_DTYPE)
    assert np.array_equal(got["seg_idx"], want["seg_idx"]) and np.array_equal(got["rec_off"], want["rec_off"])


@pytest.mark.gpu
def test_kvs_open_falls_back_when_hbm_is_short(gctx, tmp_path, monkeypatch):
    """kvr_ingest_begin answering KVR_ENOMEM (the store does not fit the HBM budget, lowered here
    by KVR_INGEST_LIMIT) switches kvs_open to the batched replay + host fold, with the same index."""
    spec = K.GenSpec(seed=103, seg_bytes=500_000, key_space_log2=11, val_min=0, val_max=300, del_permille=250)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(5)]
    ids = [1, 2, 3, 4, 5]
    d = tmp_path / "db"
    _write_store(d, segs, ids)
    want, nk, tb = expect(segs, ids)
    monkeypatch.setenv("KVR_INGEST_LIMIT", "100000")
    s = K.KVStore.open(str(d), gctx)
    assert s.open_stats().path == K.PATH_HOST_FOLD
    assert (s.stats().num_keys, s.stats().total_bytes) == (nk, tb)
    for t, k in list(zip(want, keys_of(segs, want)))[::7]:
        assert s.locate(k) == (ids[t["seg_idx"]], t["rec_off"] + 9 + t["key_len"], t["val_len"])
    s.close()
    monkeypatch.delenv("KVR_INGEST_LIMIT")
    s = K.KVStore.open(str(d), gctx)
    assert s.open_stats().path == K.PATH_DEVICE_INDEX and s.stats().num_keys == nk
    s.close()


@pytest.mark.gpu
def test_live_replay_ends_a_staged_compaction(gctx):
    """kvr_compact_stage's state shares the fold buffers: a live replay on the same context in
    between ends it, and export then answers KVR_EINVAL instead of exporting stale candidates."""
    torch = pytest.importorskip("torch")
    spec = K.GenSpec(seed=105, seg_bytes=200_000, key_space_log2=9, val_min=0, val_max=100, del_permille=200)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(3)]
    counts, kb = gctx.compact_stage(segs, [0, 1, 2], 1)
    hdr = torch.zeros(int(counts.sum()) * K.CAND_BYTES + 64, dtype=torch.uint8, device="cuda")
    keys = torch.zeros(int(kb.sum()) + 64, dtype=torch.uint8, device="cuda")
    gctx.compact_export(hdr.data_ptr(), keys.data_ptr())   # staged: fine
    gctx.replay_live(segs)
    with pytest.raises(K.NativeError, match="-1"):
        gctx.compact_export(hdr.data_ptr(), keys.data_ptr())


@pytest.mark.gpu
def test_live_keys_invalid_after_a_later_replay(gctx):
    """kvr_live_keys reads the live list of the last replay_live / replay_index; a later
    kvr_replay or kvr_compact on the same context replaces the segment descriptors and the pool,
    so the key arena must answer KVR_EINVAL rather than read stale tuples."""
    spec = K.GenSpec(seed=106, seg_bytes=200_000, key_space_log2=9, val_min=0, val_max=100, del_permille=200)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(3)]
    idx = gctx.replay_index(segs)
    keys, offs = gctx.live_keys(len(idx.live))
    assert len(offs) == len(idx.live) + 1
    gctx.replay(segs[:1])
    with pytest.raises(K.NativeError, match="-1"):
        gctx.live_keys(len(idx.live))
    idx = gctx.replay_index(segs)
    gctx.compact(segs)
    with pytest.raises(K.NativeError, match="-1"):
        gctx.live_keys(len(idx.live))


@pytest.mark.gpu
def test_kvs_open_more_segments_than_descriptors(gctx, tmp_path):
    """A store with more segment files than the process may hold descriptors (one per reopen
    over a long life, or after compactions) opens: kvs_open_ex closes each file before the next
    (engine.rs:80 opens one at a time), on the mmap and the pread path."""
    import resource
    spec = K.GenSpec(seed=107, seg_bytes=3000, key_space_log2=8, val_min=0, val_max=60, del_permille=200)
    n = 300
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(n)]
    ids = list(range(1, n + 1))
    d = tmp_path / "db"
    _write_store(d, segs, ids)
    want, nk, tb = expect(segs, ids)
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    in_use = len(os.listdir("/proc/self/fd"))
    resource.setrlimit(resource.RLIMIT_NOFILE, (in_use + 64, hard))
    try:
        for flags in (0, K.OPEN_PREAD):
            s = K.KVStore.open(str(d), gctx, flags=flags)
            assert (s.stats().num_keys, s.stats().total_bytes, s.stats().active_segment_id) == (nk, tb, n + 1)
            s.close()
            os.unlink(d / f"segment-{n + 1}.dat")
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, K.OPEN_PREAD, K.OPEN_PREAD | K.OPEN_NO_PIN])
def test_kvs_open_vanished_segment(gctx, tmp_path, monkeypatch, flags):
    """A segment file that disappears between discovery and the read (engine.rs:80-83 would fail
    its open; the knob swaps in a path that does not exist, it deletes nothing): kvs_open_ex
    answers KVR_EIO after the segments pushed before it were queued for DMA,
    and it waits for those copies (kvr_ingest_abort) before it unmaps the host bytes they read.
    The context stays usable: the same store opens cleanly once the knob is off."""
    spec = K.GenSpec(seed=108, seg_bytes=8 << 20, key_space_log2=14, val_min=0, val_max=2000, del_permille=100)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(8)]
    ids = list(range(1, 9))
    d = tmp_path / "db"
    _write_store(d, segs, ids)
    keep = bytes(segs[5])
    monkeypatch.setenv("KVS_TEST_VANISH", "5")
    with pytest.raises(K.NativeError, match=str(K.EIO)):
        K.KVStore.open(str(d), gctx, flags=flags)
    assert (d / "segment-6.dat").read_bytes() == keep   # (the knob never deletes a file)
    monkeypatch.delenv("KVS_TEST_VANISH")
    for f in d.glob("segment-9.dat"):
        f.unlink()
    want, nk, tb = expect(segs, ids)
    s = K.KVStore.open(str(d), gctx, flags=flags)
    assert (s.stats().num_keys, s.stats().total_bytes) == (nk, tb)
    s.close()
