"""k_piece, the piece mode, against the CPU oracle through the C ABI.

A stripe that starts with a run of SETs of one key and one value length is replayed value-aligned:
every value cut into 128-B pieces that end at its last byte, one piece per lane, the record headers
verified in groups against the prediction.  The first record that differs (another length, a DEL,
a bad opcode, a key with a byte >= 0x80, a segment cut) hands the stripe to k_replay's tile loop at
that record, which reports any error with every engine.rs check (src/store/engine.rs:85-151).
Every tuple field and the first error (kind, segment, offset, aux) must equal the oracle's.
"""
import functools

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

pytestmark = pytest.mark.gpu


def rec_set(k, v):
    return b"\x00" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v


def rec_del(k):
    return b"\x01" + len(k).to_bytes(4, "little") + k


def check_parity(ctx, segs, expected=None):
    ro = O.replay(segs, expected=expected)
    rg = ctx.replay(segs, expected=expected)
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


def _key(i, klen, unit=b""):
    """Record i's key of klen bytes: ASCII, or the UTF-8 character `unit` repeated (klen a multiple
    of its length)."""
    if unit:
        return unit * (klen // len(unit))
    return (b"k%011d" % i * 4)[:klen]


@functools.lru_cache(maxsize=None)
def _value(i, vlen):
    rnd = np.random.default_rng(i)
    return rnd.integers(0, 256, vlen, dtype=np.uint8).tobytes()


# keys of klen bytes with one UTF-8 failure of each kind (Rust Utf8Error: valid_up_to, error_len)
BAD_UTF8 = {
    "byte_ff": b"\xff",                       # not a lead byte (error_len 1)
    "surrogate": b"\xed\xa0\x80",             # U+D800 (error_len 1)
    "overlong": b"\xc0\x80",                  # overlong NUL (error_len 1)
    "second": b"\xe2\x28\xa1",                # 2nd byte not a continuation (error_len 1)
    "third": b"\xe2\x82\x28",                 # 3rd byte (error_len 2)
    "fourth": b"\xf0\x9f\x98\x28",            # 4th byte (error_len 3)
    "truncated": b"\xf0\x9f\x98",             # a sequence cut by the key end (error_len None)
}


def _uniform(n_rec, klen, vlen, unit=b"", change=None):
    """n_rec SETs of one key and value length; change = (i, kind) alters record i."""
    out = bytearray()
    for i in range(n_rec):
        k, v = _key(i, klen, unit), _value(i, vlen)
        if change and change[0] == i:
            kind = change[1]
            if kind in BAD_UTF8:
                bad = BAD_UTF8[kind]
                k = (k[: klen - len(bad)] + bad) if kind == "truncated" else (k[:2] + bad + k[2 + len(bad):])[:klen]
            elif kind == "utf8_ok":
                k = (k[:2] + "é".encode() + k[4:])[:klen]
            elif kind == "vlen":
                v = v[: vlen - 5]
            elif kind == "klen":
                k = k + b"z"
            elif kind == "del":
                out += rec_del(k)
                continue
            elif kind == "opcode":
                out += b"\x02" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v
                continue
            elif kind == "keylen_huge":
                out += b"\x00" + (1 << 30).to_bytes(4, "little") + k
                continue
        out += rec_set(k, v)
    return bytes(out)


# (key length, value length): P = ceil(v / 128) pieces a value, the first of r = v - 128 (P - 1)
# bytes; keys up to 36 B are read from the 48-B header window
SHAPES = [(16, 1024), (0, 128), (1, 129), (7, 200), (24, 1000), (33, 4096), (36, 8192), (5, 10000),
          (16, 65536), (37, 1024), (16, 127), (3, 131072), (9, 300000)]   # (300 KB: entries past KVR_PSEARCH tiles)


@pytest.mark.parametrize("tps", [0, 2, 8, 64])
@pytest.mark.parametrize("shape", SHAPES, ids=[f"k{k}v{v}" for k, v in SHAPES])
def test_piece_shapes(gctx, shape, tps):
    """Equal records of every piece geometry (one piece, a one-byte first piece, values of 64 and
    more pieces, keys at the window's limit and past it, values below KVR_UMIN), over stripes of
    2 to 64 tiles and the automatic layout, and a second segment of another shape behind it.  With
    300-KB values most stripes start inside a value more than KVR_PSEARCH tiles from the next record:
    k_piece hands the entry search on to k_replay."""
    klen, vlen = shape
    n_rec = max(8, (2_400_000 if vlen < 60000 else 6_000_000) // (9 + klen + vlen))
    segs = [_uniform(n_rec, klen, vlen), _uniform(300, 9, 1500)]
    gctx.set_tiles_per_stripe(tps)
    try:
        check_parity(gctx, segs)
    finally:
        gctx.set_tiles_per_stripe(0)


CHANGES = ["del", "vlen", "klen", "opcode", "utf8_ok", "keylen_huge"] + list(BAD_UTF8)


@pytest.fixture(params=["piece", "tiles"])
def engine(request, monkeypatch):
    """piece: k_piece first (the default pipeline); tiles: k_replay's tile loop alone
    (KVR_NO_PIECE=1), whose lane-parallel stride round takes the same equal records."""
    if request.param == "tiles":
        monkeypatch.setenv("KVR_NO_PIECE", "1")
    return request.param


@pytest.mark.parametrize("tps", [0, 16])
@pytest.mark.parametrize("change", CHANGES)
def test_piece_hand_back(gctx, change, tps, engine):
    """A record not as predicted at several indices of a run -- the first record, inside the first
    group, at group boundaries (63, 64, 65), deep in a stripe: k_piece hands the stripe back at
    that record (with the records of its tile already emitted) and k_replay gives the oracle's
    tuples, or its first error with aux for every UTF-8 failure kind.  The same stores through
    k_replay alone (engine "tiles")."""
    n_rec = 2300                                        # ~2.4 MB of 1033-B records
    gctx.set_tiles_per_stripe(tps)
    try:
        for i in [0, 1, 7, 63, 64, 65, 530, 2299]:
            segs = [_uniform(n_rec, 20, 1004, change=(i, change)), _uniform(200, 20, 1004)]
            check_parity(gctx, segs)
    finally:
        gctx.set_tiles_per_stripe(0)


@pytest.mark.parametrize("unit", ["é", "€", "😀"])
def test_piece_multibyte_keys(gctx, unit, engine):
    """Equal-length keys of valid 2-, 3- and 4-byte UTF-8 (the key's high bytes send the stripe to
    k_replay's full UTF-8 check), and the same with one invalid sequence mid-store."""
    u = unit.encode()
    klen = 12
    segs = [_uniform(2000, klen, 1100, unit=u)]
    check_parity(gctx, segs)
    bad = bytearray(segs[0])
    rec = 9 + klen + 1100
    pos = 777 * rec + 5 + len(u)                        # record 777's second character
    bad[pos] = 0x41                                     # a lead byte followed by ASCII
    check_parity(gctx, [bytes(bad)])


@pytest.mark.parametrize("where", ["value", "header", "key"])
def test_piece_truncated(gctx, where, engine):
    """A segment cut inside the run's last record (its value, its header, its key): the record
    does not fit, k_piece hands back there and k_replay reports engine.rs's VAL / KEY_LEN / KEY."""
    seg = _uniform(2100, 16, 1024)
    rec = 9 + 16 + 1024
    for i in [3, 1500, 2099]:
        cut = i * rec + {"value": 600, "header": 3, "key": 11}[where]
        check_parity(gctx, [seg[:cut], _uniform(50, 16, 1024)])


@pytest.mark.parametrize("klen", [25, 36, 37, 64, 300])
@pytest.mark.parametrize("bad", [None, "surrogate", "fourth", "truncated"])
def test_long_keys(gctx, klen, bad, engine):
    """Equal records with keys past the 16-B records fast path and the 36-B window (up to 300 B),
    valid and with a UTF-8 failure 700 records in: the oracle's tuples or first error with aux."""
    segs = [_uniform(1500, klen, 1000, change=(700, bad) if bad else None)]
    check_parity(gctx, segs)


def test_piece_many_chunks(gctx):
    """Short equal records in long stripes: a stripe's run takes several pool chunks (2048 slots
    each; a fresh chunk only where a tile starts), checked tuple for tuple, with the manifest."""
    n_rec = 40000                                       # 137-B records, 5.5 MB
    seg = _uniform(n_rec, 0, 128)
    man = np.array([0] * n_rec, dtype=np.uint32)
    ro = O.replay([seg])
    man[:] = ro[1]["crc32"]
    man[17] ^= 1
    gctx.set_tiles_per_stripe(256)
    try:
        rg = check_parity(gctx, [seg], expected=man)
        assert int(np.count_nonzero(rg.tuples["flags"] & K.TF_CRC_FAIL)) == 1
    finally:
        gctx.set_tiles_per_stripe(0)


def test_piece_off_matches(gctx, monkeypatch):
    """KVR_NO_PIECE=1 (k_replay alone) gives the same tuples as k_piece + k_replay."""
    segs = [_uniform(1500, 16, 1024), _uniform(1200, 16, 1024, change=(600, "del")), _uniform(400, 5, 300)]
    a = gctx.replay(segs)
    monkeypatch.setenv("KVR_NO_PIECE", "1")
    b = gctx.replay(segs)
    monkeypatch.delenv("KVR_NO_PIECE")
    assert a.status == b.status == 0 and np.array_equal(a.tuples, b.tuples)


def test_piece_index_and_keys(gctx):
    """The fold's key prefixes (kpool) from k_piece's windows: the device index of a uniform store
    equals the oracle's fold (keys repeat, so later records overwrite earlier ones)."""
    segs = []
    for s in range(3):
        out = bytearray()
        for i in range(1500):
            out += rec_set(b"key-%05d-%d" % ((i * 7 + s) % 900, s % 2), _value(i + 1000 * s, 1024))
        segs.append(bytes(out))
    ix = gctx.replay_index(segs)
    rc, t, _ = O.replay(segs)
    live, nk, _ = O.fold_live(segs, t)
    assert rc == 0 and len(ix.live) == nk and np.array_equal(ix.live, t[live])


# ---- k_piece at device bases of every alignment (KVR_SEGS_ON_DEVICE: the caller's pointers) ----
ALIGN_SHAPES = [(16, 1024), (0, 128), (36, 8192), (16, 65536)]


def _dev_place(segs, base_off):
    """Copy segs into one device buffer, segment i at an address = base_off (mod 256)."""
    torch = pytest.importorskip("torch")
    tot = sum((len(s) + 511) & ~255 for s in segs) + 512
    buf = torch.zeros(tot, dtype=torch.uint8, device="cuda")
    ptrs, off = [], base_off
    for s in segs:
        if len(s):
            buf[off: off + len(s)] = torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()).cuda()
        ptrs.append((buf.data_ptr() + off, len(s)))
        off = ((off + len(s) + 255) & ~255) + base_off
    torch.cuda.synchronize()
    return buf, ptrs


def check_parity_dev(ctx, segs, base_off):
    buf, ptrs = _dev_place(segs, base_off)
    assert all(p % 256 == base_off % 256 for p, _ in ptrs)
    ro = O.replay(segs)
    rg = ctx.replay(ptrs, on_device=True)
    assert rg.status == ro[0], (base_off, rg.status, ro[0], ro[2].kind, ro[2].rec_off)
    if ro[0] == 0:
        a, b = rg.tuples, ro[1]
        assert rg.n == len(b)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:5]
            raise AssertionError(f"base+{base_off}: tuple mismatch at {bad}: gpu={a[bad]} oracle={b[bad]}")
    else:
        eo, eg = ro[2], rg.error
        assert (eg.kind, eg.seg_idx, eg.rec_off, eg.aux) == (eo.kind, eo.seg_idx, eo.rec_off, eo.aux), base_off
    del buf


@functools.lru_cache(maxsize=None)
def _align_store(klen, vlen):
    """Uniform segments of one shape: clean, and with a record not as predicted (a DEL, another
    value length) at records 0, 64 and 530 (every index inside the store)."""
    n_rec = max(600, 2_400_000 // (9 + klen + vlen))
    segs = [_uniform(n_rec, klen, vlen)]
    for i, kind in [(0, "del"), (64, "vlen"), (530, "del")]:
        segs.append(_uniform(n_rec, klen, vlen, change=(i, kind)))
    return segs


@pytest.mark.parametrize("tps", [0, 2, 64])
@pytest.mark.parametrize("shape", ALIGN_SHAPES, ids=[f"k{k}v{v}" for k, v in ALIGN_SHAPES])
@pytest.mark.parametrize("base_off", [1, 2, 3, 5, 13, 255])
def test_piece_device_alignment(gctx, shape, tps, base_off, engine):
    """Uniform stores replayed from device buffers whose base is base_off bytes past a 256-B
    boundary (SegDesc.d0 and the piece windows' dword realignment at every residue): clean, with
    hand-backs at records 0, 64 and 530, and cut inside the last record (the first error).  The
    tiles of a stripe and k_piece's hand-back tile depend on the base, so each case runs over
    stripes of 2 and 64 tiles and the automatic layout, under both engines."""
    klen, vlen = shape
    segs = _align_store(klen, vlen)
    gctx.set_tiles_per_stripe(tps)
    try:
        check_parity_dev(gctx, list(segs), base_off)
        cut = segs[0][: len(segs[0]) - (vlen // 2)]        # the last record's value cut in half
        check_parity_dev(gctx, [segs[1], cut], base_off)
    finally:
        gctx.set_tiles_per_stripe(0)


def test_piece_adaptive_skip(gctx):
    """A device-resident store that k_piece hands back entirely (values of 1000 and 1001 B alternating:
    no stripe starts a run of equal records) makes the library skip k_piece on the next calls with
    the same segment layout (KVR_PIECE_ADAPT).  The tuples never depend on it: the same buffer then
    refilled with a uniform store of the same length replays to the oracle's tuples whether k_piece
    runs or not, call after call."""
    torch = pytest.importorskip("torch")
    a = bytearray()
    for i in range(2000):
        a += rec_set(_key(i, 16), _value(i, 1000 + (i & 1)))
    b = bytearray()
    for i in range(1000):
        b += rec_set(_key(i, 16), _value(i, 2051 - 25))
    assert len(a) == len(b)
    buf = torch.zeros(len(a) + 512, dtype=torch.uint8, device="cuda")
    ptrs = [(buf.data_ptr() + 64, len(a))]
    for store in (bytes(a), bytes(b)):
        buf[64: 64 + len(store)] = torch.from_numpy(np.frombuffer(store, dtype=np.uint8).copy()).cuda()
        torch.cuda.synchronize()
        rc, ref, _ = O.replay([store])
        assert rc == 0
        for _ in range(10):
            rg = gctx.replay(ptrs, on_device=True)
            assert rg.status == 0 and np.array_equal(rg.tuples, ref)
