"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle, bit-exact.

Every tuple field (rec_off, seg_idx, key_len, val_len, crc32, key_tag, op, flags) and every
error (kind, segment, offset, aux) must equal the oracle's on the same bytes.
"""
import os
import random
import shutil
import zlib

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
KIND = {"NONE": 0, "OPEN": 1, "KEY_LEN": 2, "KEY": 3, "UTF8": 4, "VAL_LEN": 5, "VAL": 6, "OPCODE": 7}


def rec_set(k, v):
    return b"\x00" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v


def rec_del(k):
    return b"\x01" + len(k).to_bytes(4, "little") + k


def read_dir(name):
    d = os.path.join(GOLD, name)
    names = sorted((n for n in os.listdir(d) if n.startswith("segment-")), key=lambda n: int(n[8:-4]))
    return [int(n[8:-4]) for n in names], [open(os.path.join(d, n), "rb").read() for n in names]


def check_parity(ctx, segs, expected=None, seg_ids=None):
    ro = O.replay(segs, expected=expected, seg_ids=seg_ids)
    rg = ctx.replay(segs, seg_ids=seg_ids, expected=expected)
    assert rg.status == ro[0], (rg.status, ro[0], ro[2].kind, ro[2].rec_off)
    if ro[0] == 0:
        assert rg.n == len(ro[1])
        a, b = rg.tuples, ro[1]
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:5]
            raise AssertionError(f"tuple mismatch at {bad}: gpu={a[bad]} oracle={b[bad]}")
    else:
        eo, eg = ro[2], rg.error
        assert (eg.kind, eg.seg_idx, eg.rec_off, eg.aux) == (eo.kind, eo.seg_idx, eo.rec_off, eo.aux)
    return rg


@pytest.mark.parametrize("name", ["persistence", "store_integration", "compaction_example", "large_dataset"])
def test_golden_dirs(gctx, name):
    ids, segs = read_dir(name)
    check_parity(gctx, segs, seg_ids=ids)
    if name == "persistence":   # config 1: replay of segment-1 alone
        check_parity(gctx, segs[:1], seg_ids=ids[:1])


def test_negative_cases(gctx, golden):
    for c in golden["negative"]:
        data = bytes.fromhex(c["hex"])
        rg = check_parity(gctx, [data])
        if c["kind"] != "NONE":
            assert rg.error.kind == KIND[c["kind"]], c["name"]
        # the same failure behind a good segment, and with the bad one first
        check_parity(gctx, [read_dir("store_integration")[1][0], data])
        check_parity(gctx, [data, read_dir("compaction_example")[1][0]])


SPECS = {
    "cfg2_1k": K.GenSpec(seed=21, seg_bytes=700_000, val_min=1024, val_max=1024),
    "cfg3_64k": K.GenSpec(seed=31, seg_bytes=1_500_000, val_min=65536, val_max=65536),
    "cfg4_del": K.GenSpec(seed=41, seg_bytes=600_000, val_min=1024, val_max=1024, del_permille=500),
    "cfg5_zipf": K.GenSpec(seed=51, seg_bytes=3_000_000, key_dist=1, key_space_log2=24, val_min=16,
                           val_max=1 << 20, del_permille=100),
    "tiny": K.GenSpec(seed=61, seg_bytes=200_000, val_min=0, val_max=40, del_permille=300),
    "flips": K.GenSpec(seed=71, seg_bytes=400_000, val_min=16, val_max=9000, flip_per_million=50_000),
}


@pytest.mark.parametrize("name", list(SPECS))
def test_generated_parity(gctx, name):
    spec = SPECS[name]
    segs, exps = zip(*[K.gen_segment_cpu(spec, s) for s in range(3)])
    exp = np.concatenate(exps)
    rg = check_parity(gctx, list(segs), expected=exp)
    if name == "flips":
        assert rg.stats.n_crc_fail > 0
        assert rg.stats.n_crc_fail == int(np.sum((rg.tuples["flags"] & K.TF_CRC_FAIL) != 0))
    else:
        assert rg.stats.n_crc_fail == 0


@pytest.mark.parametrize("tps", [2, 5, 64, 100000])
@pytest.mark.parametrize("name", ["cfg2_1k", "cfg3_64k", "cfg4_del", "cfg5_zipf", "tiny", "flips"])
def test_multi_tile_stripes(gctx, name, tps):
    """Stripes of several tiles: exact chains across tiles, carried values, stripe speculation."""
    spec = SPECS[name]
    segs, exps = zip(*[K.gen_segment_cpu(spec, s) for s in range(3)])
    gctx.set_tiles_per_stripe(tps)
    try:
        check_parity(gctx, list(segs), expected=np.concatenate(exps))
    finally:
        gctx.set_tiles_per_stripe(0)


def boundary_segment(tile=16384):
    """Records whose start sits at every offset r in [-44, 8] around a tile boundary, for several
    key and value lengths: headers, key bytes, length fields and the first value bytes straddle
    the boundary in every possible way (fillers align each probe record)."""
    out = bytearray()
    for klen in (0, 3, 16):
        for vlen in (0, 5, 64, 65, 200, 20000):
            for r in range(-44, 9):
                b = (len(out) // tile + 2) * tile
                fill = b + r - len(out) - 10                  # filler: 9 + 1 (key "f") + fill bytes
                out += rec_set(b"f", bytes((len(out) + j) & 255 for j in range(fill)))
                assert len(out) == b + r
                out += rec_set(bytes(97 + j % 26 for j in range(klen)), bytes((r * 7 + j) & 255 for j in range(vlen)))
    out += rec_del(b"end")
    return bytes(out)


def test_tile_boundary_sweep(gctx):
    seg = boundary_segment()
    rc, ref, _ = O.replay([seg])
    assert rc == 0
    for tps in (0, 1, 4):
        gctx.set_tiles_per_stripe(tps)
        try:
            check_parity(gctx, [seg, seg[:-3]])
        finally:
            gctx.set_tiles_per_stripe(0)
    torch = pytest.importorskip("torch")
    buf = torch.zeros(len(seg) + 64, dtype=torch.uint8, device="cuda")
    for shift in (1, 5, 13):                           # device placement moves the tile grid
        buf.zero_()
        buf[shift: shift + len(seg)] = torch.frombuffer(bytearray(seg), dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        for tps in (0, 3):
            gctx.set_tiles_per_stripe(tps)
            rg = gctx.replay([(buf.data_ptr() + shift, len(seg))], on_device=True)
            gctx.set_tiles_per_stripe(0)
            assert rg.status == 0 and np.array_equal(rg.tuples, ref), (shift, tps)


def test_adversarial_speculation(gctx):
    """Values that look like records defeat the speculative entry; results must stay exact."""
    inner = b"".join(rec_set(b"k%d" % i, b"v" * (i % 50)) for i in range(4000))       # a segment in a value
    zeros = bytes(200_000)                                                              # 9-byte empty SETs
    rng = random.Random(5)
    parts = []
    for i in range(60):
        kind = i % 3
        v = inner if kind == 0 else zeros if kind == 1 else bytes(rng.getrandbits(8) for _ in range(3000))
        parts.append(rec_set(b"key%d" % i, v[: rng.randint(1, len(v))]))
        if i % 7 == 0:
            parts.append(rec_del(b"key%d" % (i // 2)))
    seg = b"".join(parts)
    check_parity(gctx, [seg, seg[: len(seg) // 2 + 13], inner, zeros])


def test_pool_overflow_retry(gctx):
    """Records far denser than the pool estimate (5-byte DELs of empty keys, few long stripes):
    the waves' claims run past the pool, land in its slack, the overflow is flagged, and the host
    grows the pool and replays again -- same tuples as the oracle (engine.rs:139-141 DEL records)."""
    dense = rec_del(b"") * ((8 << 20) // 5)
    mixed = b"".join(rec_set(b"k%d" % i, b"") + rec_del(b"") * 7 for i in range(100_000))
    gctx.set_tiles_per_stripe(1024)
    try:
        check_parity(gctx, [dense, mixed, dense[:-2]])
        check_parity(gctx, [mixed, dense])
    finally:
        gctx.set_tiles_per_stripe(0)


def _blob_store(image_values, seed):
    """A segment whose big values are whole segment images (valid record chains), each spanning
    hundreds of single-tile stripes, between runs of ordinary records."""
    rng = random.Random(seed)
    parts = []
    for i, v in enumerate(image_values):
        for j in range(200):
            parts.append(rec_set(b"k%d.%d" % (i, j), bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 300)))))
        parts.append(rec_set(b"blob%d" % i, v))
    parts.append(rec_del(b"k0.0"))
    return b"".join(parts)


def test_adversarial_walk_through(gctx):
    """Every stripe inside a value that holds a segment image speculates an entry on the image's
    records, and those stripes agree with each other.  k_link lists only the first stripe of such
    a run and its re-walk walks on through the rest (engine.rs:85-151 chain), so the store
    replays in one re-walk round instead of one per stripe; timed against a store of the same
    shape whose big values are random bytes (no wrong speculation)."""
    import time
    rng = random.Random(17)
    image = b"".join(rec_set(b"in%d" % i, bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 90))))
                     for i in range(30000))                    # ~1.8 MiB of valid records
    images = [image, image[: len(image) // 2]]
    noise = [bytes(rng.getrandbits(8) for _ in range(len(v))) for v in images]
    adv, clean = _blob_store(images, 3), _blob_store(noise, 3)
    assert len(adv) == len(clean)
    gctx.set_tiles_per_stripe(1)                               # ~350 stripes inside the big values
    try:
        rg = check_parity(gctx, [adv, adv[: len(adv) - 7]])
        check_parity(gctx, [adv])
        st = gctx.last_stats()
        n_redo_adv = st.n_redo
        check_parity(gctx, [clean])
        n_redo_clean = gctx.last_stats().n_redo

        def best(seg):
            t = []
            for _ in range(3):
                t0 = time.perf_counter()
                r = gctx.replay([seg])
                t.append(time.perf_counter() - t0)
                assert r.status == 0
            return min(t)
        ta, tc = best(adv), best(clean)
    finally:
        gctx.set_tiles_per_stripe(0)
    print(f"adversarial: n_redo {n_redo_adv} {ta * 1e3:.2f} ms; clean: n_redo {n_redo_clean} {tc * 1e3:.2f} ms")
    assert n_redo_adv <= 2, n_redo_adv
    assert ta <= 2.0 * tc + 2e-3, (ta, tc)


def test_random_truncations_and_corruptions(gctx):
    spec = K.GenSpec(seed=81, seg_bytes=400_000, val_min=1, val_max=3000, del_permille=200)
    base, _ = K.gen_segment_cpu(spec, 0)
    base = base.tobytes()
    rc, t, _ = O.replay([base])
    offs = t["rec_off"].astype(np.int64)
    rng = random.Random(9)
    for trial in range(24):
        b = bytearray(base)
        mode = trial % 4
        j = rng.randrange(len(offs))
        o = int(offs[j])
        if mode == 0:
            b = b[: o + rng.randint(1, 40)]                  # torn tail inside a record
        elif mode == 1:
            b[o] = rng.choice([2, 3, 0x7F, 0xFF])            # bad opcode
        elif mode == 2:
            b[o + 5 + rng.randrange(16)] = 0xFF              # invalid UTF-8 in a key
        else:
            b[o + 1: o + 5] = (len(b)).to_bytes(4, "little")  # key length past the end
        good, _ = K.gen_segment_cpu(spec, 1)
        check_parity(gctx, [good.tobytes(), bytes(b), good.tobytes()])


def test_device_segments_at_odd_alignment(gctx):
    torch = pytest.importorskip("torch")
    spec = SPECS["cfg5_zipf"]
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(3)]
    rc, ref, _ = O.replay(segs)
    buf = torch.zeros(sum(len(s) for s in segs) + 4096, dtype=torch.uint8, device="cuda")
    ptrs, off = [], 3
    for s in segs:
        buf[off: off + len(s)] = torch.from_numpy(s).cuda()
        ptrs.append((buf.data_ptr() + off, len(s)))
        off += len(s) + 7
    torch.cuda.synchronize()
    rg = gctx.replay(ptrs, on_device=True)
    assert rg.status == 0 and np.array_equal(rg.tuples, ref)


def test_device_generator_matches_cpu(gctx):
    torch = pytest.importorskip("torch")
    for spec in (SPECS["cfg5_zipf"], SPECS["flips"], SPECS["cfg4_del"]):
        for seg_no in (0, 3):
            b, e = K.gen_segment_cpu(spec, seg_no)
            d = torch.zeros(len(b) + 64, dtype=torch.uint8, device="cuda")
            de = torch.zeros(len(e) + 4, dtype=torch.int32, device="cuda")
            ln, nr = gctx.gen_segment_device(spec, seg_no, d.data_ptr(), d.numel(), de.data_ptr(), de.numel())
            torch.cuda.synchronize()
            assert (ln, nr) == (len(b), len(e))
            assert np.array_equal(d[:ln].cpu().numpy(), b)
            assert np.array_equal(de[:nr].cpu().numpy().view(np.uint32), e)


def test_kvstore_open_golden(gctx, tmp_path):
    d = tmp_path / "persisted_store"
    shutil.copytree(os.path.join(GOLD, "persistence"), d)
    s = K.KVStore.open(str(d), gctx)
    assert s.get("session") == b"first" and s.get("counter") == b"43" and s.get("name") is None
    assert s.locate("counter") == (2, 16, 2)
    st = s.stats()
    assert (st.num_keys, st.total_bytes, st.active_segment_id) == (2, 7, 4)
    assert st.num_segments == 4                       # segment-1..3 + the new active segment-4
    s.close()
    d2 = tmp_path / "large"
    shutil.copytree(os.path.join(GOLD, "large_dataset"), d2)
    s = K.KVStore.open(str(d2), gctx)
    assert s.get("user:05000:data") == b"User data for ID 5000" and s.stats().num_keys == 10000
    s.close()


def test_kvstore_open_reports_reference_message(gctx, tmp_path):
    d = tmp_path / "db"
    d.mkdir()
    (d / "segment-1.dat").write_bytes(rec_set(b"a", b"1"))
    (d / "segment-2.dat").write_bytes(rec_set(b"b", b"2") + b"\x00\x05\x00")
    with pytest.raises(K.CorruptedData) as ei:
        K.KVStore.open(str(d), gctx)
    assert str(ei.value) == f"Corrupted data: Failed to read key length in {d}/segment-2.dat: failed to fill whole buffer"


def test_sharded_replay_matches_single(gctx):
    """N-way round-robin sharding (two contexts on one device stand in for two GPUs) merges back
    into exactly the single-context answer, including the store's first error."""
    from kvreplay import shard as SH
    spec = SPECS["cfg4_del"]
    parts = [K.gen_segment_cpu(spec, s) for s in range(5)]
    segs = [p[0] for p in parts]
    ctx2 = K.Context(0)
    try:
        sr = SH.ShardedReplay(contexts=[gctx, ctx2])
        st, t, err = sr.replay(segs)
        rc, ref, _ = O.replay(segs)
        assert st == rc == 0 and np.array_equal(t, ref)
        exp = (np.concatenate([p[1] for p in parts]), [len(p[1]) for p in parts])
        st, t, _ = sr.replay(segs, expected=exp)
        assert st == 0 and not np.any(t["flags"] & K.TF_CRC_FAIL) and np.all(t["flags"][t["op"] == 0] & 1)
        bad = [s.tobytes() for s in segs]
        bad[2], bad[3] = bad[2][:-5], bad[3][:-2]
        st, _, err = sr.replay(bad)
        rc, _, e = O.replay(bad)
        assert st == rc == 1 and err == (e.kind, e.seg_idx, e.rec_off, e.aux) and err[1] == 2
    finally:
        ctx2.close()


def test_segment_over_2gib(gctx):
    """Maximum sizes: a segment that runs more than 2 GiB past its tiles (the 64-bit copy of the
    hop loop) holding a value larger than 2 GiB, with ordinary records on both sides, and a
    second segment after it; plus the same segment cut short inside the big value (KVR_E_VAL)."""
    big = (1 << 31) + 12345
    head = b"".join(rec_set(f"k{i}".encode(), bytes([i]) * (i * 37 % 300)) for i in range(200))
    tail = b"".join(rec_set(f"t{i}".encode(), bytes([255 - i]) * (i * 53 % 900)) for i in range(200)) + rec_del(b"k3")
    seg = np.empty(len(head) + 9 + 3 + big + len(tail), dtype=np.uint8)
    o = 0
    seg[o: o + len(head)] = np.frombuffer(head, np.uint8); o += len(head)
    hdr = b"\x00" + (3).to_bytes(4, "little") + b"big" + big.to_bytes(4, "little")
    seg[o: o + len(hdr)] = np.frombuffer(hdr, np.uint8); o += len(hdr)
    seg[o: o + big] = 0
    seg[o: o + big: 4099] = 0xA5                     # a sparse pattern (the CRC must see every byte)
    o += big
    seg[o: o + len(tail)] = np.frombuffer(tail, np.uint8); o += len(tail)
    assert o == len(seg)
    second = rec_set(b"k3", b"again") + rec_set(b"big", b"small now")
    check_parity(gctx, [seg, second])
    cut = seg[: len(head) + len(hdr) + big // 2]      # the big value is truncated: engine.rs:130
    rg = check_parity(gctx, [cut])
    assert rg.error.kind == KIND["VAL"]


def test_repeated_calls_reuse_and_refresh_descriptors(gctx):
    """Calls over the same segments reuse the uploaded descriptors and stripe layout; a call over
    other segments (same count, other lengths), a corrupted call (its counters are not cleared
    behind it) and the calls after it must still match the oracle bit for bit."""
    spec_a, spec_b = SPECS["cfg2_1k"], SPECS["cfg4_del"]
    a = [K.gen_segment_cpu(spec_a, s)[0].tobytes() for s in range(3)]
    b = [K.gen_segment_cpu(spec_b, s)[0].tobytes() for s in range(3)]
    bad = a[:2] + [a[2][: len(a[2]) // 2 + 7]]
    for segs in (a, a, b, a, bad, bad, a, b, b):
        check_parity(gctx, segs)


@pytest.mark.parametrize("link_kernel", [False, True])
@pytest.mark.parametrize("tps", [0, 2])
@pytest.mark.parametrize("name", ["cfg2_1k", "cfg3_64k", "cfg4_del", "cfg5_zipf", "flips"])
def test_linked_gather_and_link_kernel(gctx, monkeypatch, name, tps, link_kernel):
    """The replay pipeline's two ways to order the pool: k_compact_s linking every stripe itself
    (the default: no k_link launch; a stripe it cannot link alone sends the call to k_link), and
    k_link first (KVR_LINK_KERNEL=1).  Same tuples, CRC flags and first error; a corrupted call
    between clean ones (the double-buffered counter blocks) changes nothing after it."""
    if link_kernel:
        monkeypatch.setenv("KVR_LINK_KERNEL", "1")
    spec = SPECS[name]
    segs, exps = zip(*[K.gen_segment_cpu(spec, s) for s in range(3)])
    segs = [s.tobytes() for s in segs]
    exp = np.concatenate(exps)
    bad = segs[:2] + [segs[2][: len(segs[2]) * 2 // 3 + 5]]
    gctx.set_tiles_per_stripe(tps)
    try:
        for i, (ss, ee) in enumerate(((segs, exp), (segs, exp), (bad, None), (segs, exp))):
            rg = check_parity(gctx, ss, expected=ee)
            if ee is not None:
                assert rg.stats.n_crc_fail == int(np.sum((rg.tuples["flags"] & K.TF_CRC_FAIL) != 0))
            if link_kernel:
                assert rg.stats.n_link_passes >= 1
    finally:
        gctx.set_tiles_per_stripe(0)


def _equal_store(n_rec, klen=10, vlen=1000, change=None):
    """n_rec equal SETs (the batched speculative tiles' case: ~8 records a tile), record i's key
    and value derived from i; change = (i, kind) alters record i: 'utf8' (an invalid key byte),
    'opcode' (opcode 7), 'vlen' (a shorter value, a valid record), 'del' (a DEL instead),
    'klen' (a longer key, valid)."""
    out = bytearray()
    for i in range(n_rec):
        k = (b"k%09d" % i)[:klen].ljust(klen, b"x")
        v = bytes((i * 7 + j) & 255 for j in range(vlen))
        if change and change[0] == i:
            kind = change[1]
            if kind == "utf8":
                k = k[:3] + b"\xff" + k[4:]
            elif kind == "vlen":
                v = v[: vlen - 123]
            elif kind == "klen":
                k = k + b"yyyy"
            elif kind == "del":
                out += rec_del(k)
                continue
            if kind == "opcode":
                out += b"\x07" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v
                continue
        out += rec_set(k, v)
    return bytes(out)


@pytest.mark.parametrize("tps", [0, 8, 64])
@pytest.mark.parametrize("change", [None, "utf8", "opcode", "vlen", "del", "klen", "trunc"])
def test_batched_speculative_tiles(gctx, tps, change):
    """Equal records over long stripes: speculative tiles verify and emit the predicted records of
    the next whole tiles in one batch.  A record several tiles into a batch that is not as
    predicted (another value or key length, a DEL: valid; a bad opcode, an invalid UTF-8 key:
    errors, the latter found only by the records phase) and a segment cut mid-record must give
    the oracle's tuples or first error, at several record indices past a tile boundary."""
    n_rec = 2200                                   # ~2.2 MB: 280 tiles
    picks = [None] if change is None else [41, 97, 530, 1777]
    gctx.set_tiles_per_stripe(tps)
    try:
        for i in picks:
            if change == "trunc":
                seg = _equal_store(n_rec)
                cut = i * 1019 + 600                   # inside record i's value
                segs = [seg[:cut]]
            else:
                segs = [_equal_store(n_rec, change=None if i is None else (i, change))]
            segs = segs + [_equal_store(300)]          # a clean segment behind it
            check_parity(gctx, segs)
    finally:
        gctx.set_tiles_per_stripe(0)


def _varied_store(seed, n_bytes, del_frac, klen_rng, vlen_rng, zero_values=False, key_alphabet=None):
    """Records of varying lengths (the candidate rounds' case): keys of random length from
    key_alphabet (ASCII letters by default), values random or all zero."""
    rnd = random.Random(seed)
    alpha = key_alphabet or [bytes([c]) for c in range(0x41, 0x5B)] + [bytes([c]) for c in range(0x61, 0x7B)]
    out = bytearray()
    while len(out) < n_bytes:
        k = b"".join(rnd.choice(alpha) for _ in range(rnd.randint(*klen_rng)))
        if rnd.random() < del_frac:
            out += rec_del(k)
        else:
            n = rnd.randint(*vlen_rng)
            v = bytes(n) if zero_values else rnd.randbytes(n)
            out += rec_set(k, v)
    return bytes(out)


CAND_STORES = {
    # keys of 1 .. 40 bytes (lengths other than the first record's take the successor from memory;
    # keys past 24 bytes the long-key CRC), values up to 300 B, 30 % DEL
    "mixed_keys": dict(del_frac=0.3, klen_rng=(1, 40), vlen_rng=(0, 300)),
    # 95 % DEL of short records: a few hundred records a tile, windows of 64 candidates
    "del_heavy": dict(del_frac=0.95, klen_rng=(8, 16), vlen_rng=(0, 40)),
    # zero-valued SETs: every value byte is a candidate, so units past 64 go to the exact loop
    "zero_values": dict(del_frac=0.2, klen_rng=(4, 20), vlen_rng=(50, 3000), zero_values=True),
    # keys of control and multi-byte characters: candidates inside keys, the UTF-8 check per record
    "odd_keys": dict(del_frac=0.3, klen_rng=(1, 12), vlen_rng=(0, 200),
                     key_alphabet=[b"\x00", b"\x01", b"a", b"\xc3\xa9", b"\xe2\x82\xac", b"\xf0\x9f\x98\x80"]),
}


@pytest.mark.parametrize("tps", [0, 2])
@pytest.mark.parametrize("name", list(CAND_STORES))
def test_candidate_rounds(gctx, name, tps):
    """Stores whose record lengths vary tile to tile (the candidate-chain framing and its windows,
    k_replay), bit-exact against the oracle; the same with a broken record planted mid-segment
    (the chain breaks there and the exact loop reports engine.rs's error) and with an invalid UTF-8
    key in the middle (the first error of a candidate round by rank)."""
    kw = CAND_STORES[name]
    segs = [_varied_store(1000 * i + len(name), 250_000, **kw) for i in range(3)]
    gctx.set_tiles_per_stripe(tps)
    try:
        check_parity(gctx, segs)
        # a record start overwritten with an opcode of 7 about two thirds into segment 1
        ro = O.replay([segs[1]])
        offs = ro[1]["rec_off"]
        at = int(offs[2 * len(offs) // 3])
        bad = bytearray(segs[1])
        bad[at] = 7
        check_parity(gctx, [segs[0], bytes(bad), segs[2]])
        # an invalid UTF-8 key: the first key byte of a later record set to 0xFF (a 1-byte key
        # stays a valid record framing)
        at2 = int(offs[len(offs) // 2])
        bad2 = bytearray(segs[1])
        bad2[at2 + 5] = 0xFF if int.from_bytes(bad2[at2 + 1:at2 + 5], "little") else bad2[at2 + 5]
        check_parity(gctx, [segs[0], bytes(bad2), segs[2]])
    finally:
        gctx.set_tiles_per_stripe(0)
