"""Pin the CPU oracle (oracle/replay_ref.c) against the reference's own fixtures.

The reference (Rust) cannot be built here, so the oracle is pinned by:
  - the final maps / key counts the reference's tests and examples assert
    (examples/persistence.rs:18-37, :54-67; tests/store_integration.rs:22-31;
     examples/compaction.rs:28-35, :54-63; examples/large_dataset.rs:29-49, :76),
  - the SURVEY.md §8c segment bytes and tuple constants,
  - CRC-32/ISO-HDLC known answers (zlib.crc32 — crc32fast 1.5.0 implements the same function),
  - Python's UTF-8 decoder for Rust's Utf8Error (valid_up_to / error_len) semantics,
  - the check order of engine.rs:85-149 for the negative cases.
"""
import os
import random
import zlib

import numpy as np
import pytest

import oracle_py as O

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
KIND = {"NONE": 0, "OPEN": 1, "KEY_LEN": 2, "KEY": 3, "UTF8": 4, "VAL_LEN": 5, "VAL": 6, "OPCODE": 7}

# SURVEY.md §8c hex (independent restatement of examples/persistence.rs sessions 1 and 2)
SURVEY_SEG1 = ("000700000073657373696f6e0500000066697273740007000000636f756e74657202000000343200"
               "040000006e616d650a000000546573742053746f7265")
SURVEY_SEG2 = "0007000000636f756e74657202000000343301040000006e616d65"


def read_dir(name):
    d = os.path.join(GOLD, name)
    names = sorted((n for n in os.listdir(d) if n.startswith("segment-")), key=lambda n: int(n[8:-4]))
    return [int(n[8:-4]) for n in names], [open(os.path.join(d, n), "rb").read() for n in names]


def fold_map(segs, tuples):
    """engine.rs:137/:141 restated in Python over oracle tuples (small cases only)."""
    m = {}
    for t in tuples:
        s = segs[t["seg_idx"]]
        k = bytes(s[t["rec_off"] + 5: t["rec_off"] + 5 + t["key_len"]])
        if t["op"] == 0:
            vo = t["rec_off"] + 9 + t["key_len"]
            m[k] = (bytes(s[vo: vo + t["val_len"]]), int(t["seg_idx"]), int(t["rec_off"]), vo, int(t["crc32"]))
        else:
            m.pop(k, None)
    return m


def test_crc_known_answers(golden):
    assert O.crc32(b"123456789") == 0xCBF43926 == int(golden["crc_check"]["crc32"], 16)
    assert O.crc32(b"") == 0
    assert O.crc32(b"Hello, World!") == zlib.crc32(b"Hello, World!") == 0xEC4AC3D0   # README:174 is illustrative
    rng = random.Random(7)
    for n in list(range(0, 70)) + [255, 256, 1023, 4096, 65537]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.crc32(b) == zlib.crc32(b)
        # streaming (crc32fast::Hasher::update) == one shot
        k = n // 3
        assert O.crc32(b[k:], O.crc32(b[:k])) == zlib.crc32(b)


def _py_utf8(b):
    try:
        b.decode("utf-8")
        return True, 0, 0
    except UnicodeDecodeError as e:
        if e.reason == "unexpected end of data":
            return False, e.start, 0
        return False, e.start, e.end - e.start


def test_utf8_matches_rust_semantics_via_python():
    rng = random.Random(11)
    pool = [0x41, 0x7F, 0x80, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF, 0xE0, 0xE1, 0xEC, 0xED, 0xEE, 0xEF, 0xF0, 0xF1,
            0xF3, 0xF4, 0xF5, 0xFF, 0x9F, 0xA0, 0x8F, 0x90, 0x30]
    cases = [b"", b"abc", "é€😀ключ".encode(), b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xe0\x9f\x80",
             b"\xf0\x8f\xbf\xbf", b"\xc2", b"\xe2\x82", b"\xf0\x9f\x98", b"a\xc0\xafb"]
    for _ in range(20000):
        n = rng.randint(1, 7)
        cases.append(bytes(rng.choice(pool) for _ in range(n)))
    for c in cases:
        assert O.utf8_check(c) == _py_utf8(c), c.hex()


def test_persistence_fixture_bytes_match_survey(golden):
    ids, segs = read_dir("persistence")
    assert ids == [1, 2, 3]
    assert segs[0].hex() == SURVEY_SEG1 == golden["persistence"]["hex_segment_1"]
    assert segs[1].hex() == SURVEY_SEG2 == golden["persistence"]["hex_segment_2"]
    assert segs[2] == b""


def test_persistence_session2_replays_one_segment(golden):
    """Config 1 of BASELINE.json: replay segment-1 only (persistence.rs:17-37)."""
    ids, segs = read_dir("persistence")
    rc, t, _ = O.replay(segs[:1], seg_ids=ids[:1])
    assert rc == 0 and len(t) == 3
    m = fold_map(segs[:1], t)
    exp = golden["persistence"]["after_segment_1"]
    assert set(m) == {e[0].encode() for e in exp}
    for key, seg_id, rec_off, val_off, vlen, crc in exp:
        v, si, ro, vo, c = m[key.encode()]
        assert (ids[si], ro, vo, len(v), c) == (seg_id, rec_off, val_off, vlen, int(crc, 16))
        assert zlib.crc32(v) == c
    assert m[b"session"][0] == b"first" and m[b"counter"][0] == b"42" and m[b"name"][0] == b"Test Store"
    live, nk, tb = O.fold_live(segs[:1], t)
    assert (nk, tb) == (3, 17)


def test_persistence_session3_replays_all(golden):
    """persistence.rs:53-67: counter == 43, name deleted; segment-3 is empty (engine.rs:62-68)."""
    ids, segs = read_dir("persistence")
    rc, t, _ = O.replay(segs, seg_ids=ids)
    assert rc == 0 and len(t) == 5
    m = fold_map(segs, t)
    assert m[b"session"][0] == b"first" and m[b"counter"][0] == b"43" and b"name" not in m
    for key, seg_id, rec_off, val_off, vlen, crc in golden["persistence"]["after_all"]:
        v, si, ro, vo, c = m[key.encode()]
        assert (ids[si], ro, vo, len(v), c) == (seg_id, rec_off, val_off, vlen, int(crc, 16))
    dels = [x for x in t if x["op"] == 1]
    assert len(dels) == 1 and (ids[dels[0]["seg_idx"]], int(dels[0]["rec_off"])) == (2, 18)
    live, nk, tb = O.fold_live(segs, t)
    assert (nk, tb) == (2, 7)


@pytest.mark.parametrize("name,rounds", [("store_integration", 5), ("compaction_example", 10)])
def test_overwrite_rounds(golden, name, rounds):
    """tests/store_integration.rs:22-31 and examples/compaction.rs:28-35/:54-63."""
    g = golden[name]
    ids, segs = read_dir(name)
    assert len(segs[0]) == g["files"]["segment-1.dat"]["size"]
    assert "%08x" % zlib.crc32(segs[0]) == g["files"]["segment-1.dat"]["crc32"]
    rc, t, _ = O.replay(segs, seg_ids=ids)
    assert rc == 0 and len(t) == rounds * 100
    m = fold_map(segs, t)
    assert len(m) == 100 == g["num_keys"]
    for i in range(100):
        assert m[b"key_%d" % i][0] == b"value_%d_%d" % (i, rounds - 1)
    live, nk, tb = O.fold_live(segs, t)
    assert (nk, tb) == (g["num_keys"], g["total_bytes"])
    if name == "store_integration":
        v, si, ro, vo, c = m[b"key_0"]
        assert (ro, vo, len(v), c) == (g["key_0"]["rec_off"], g["key_0"]["val_off"], g["key_0"]["vlen"],
                                       int(g["key_0"]["crc32"], 16))
        v, si, ro, vo, c = m[b"key_99"]
        assert (ro, vo, len(v)) == (g["key_99"]["rec_off"], g["key_99"]["val_off"], g["key_99"]["vlen"])


def test_large_dataset(golden):
    """examples/large_dataset.rs:29-49 and :76 (10,000 keys)."""
    g = golden["large_dataset"]
    ids, segs = read_dir("large_dataset")
    rc, t, _ = O.replay(segs, seg_ids=ids)
    assert rc == 0 and len(t) == 10000
    m = fold_map(segs, t)
    for k, v in g["samples"].items():
        assert m[k.encode()][0] == v.encode()
    for i in range(0, 10000, 10):
        assert m[b"user:%05d:data" % i][0] == b"User data for ID %d" % i
    live, nk, tb = O.fold_live(segs, t)
    assert (nk, tb) == (10000, g["total_bytes"])


def test_negative_cases(golden):
    for c in golden["negative"]:
        data = bytes.fromhex(c["hex"])
        rc, t, err = O.replay([data])
        if c["kind"] == "NONE":
            assert rc == 0, c["name"]
            continue
        assert rc == 1, c["name"]
        assert err.kind == KIND[c["kind"]], (c["name"], err.kind)
        assert err.rec_off == c["off"] and err.seg_idx == 0, c["name"]
        if c["kind"] == "OPCODE":
            assert err.aux == c["aux"], c["name"]
        if c["kind"] == "UTF8":
            assert (err.aux & 0xFFFFFFFF, err.aux >> 32) == tuple(c["aux"]), c["name"]


def test_first_error_aborts_in_segment_order():
    """engine.rs:55-56: segments replay in id order and the first error aborts open()."""
    ok = b"\x00\x01\x00\x00\x00a\x01\x00\x00\x00b"
    bad1 = ok + b"\x05"                     # KEY_LEN at 11
    bad2 = b"\x03\x00\x00\x00\x00"          # OPCODE at 0
    rc, t, err = O.replay([ok, bad1, bad2])
    assert rc == 1 and (err.seg_idx, err.rec_off, err.kind) == (1, 11, 2)
    rc, t, err = O.replay([ok, bad2, bad1])
    assert rc == 1 and (err.seg_idx, err.rec_off, err.kind, err.aux) == (1, 0, 7, 3)


def test_faithful_baseline_agrees_with_fold():
    ids, segs = read_dir("compaction_example")
    rc, nk, tb, nr, dg, err = O.replay_faithful(segs)
    assert (rc, nk, tb, nr) == (0, 100, 990, 1000)
    ids, segs = read_dir("persistence")
    rc, nk, tb, nr, dg, err = O.replay_faithful(segs)
    assert (rc, nk, tb, nr) == (0, 2, 7, 5)
    rc, *_ , err = O.replay_faithful([bytes.fromhex("0002000000ff00")])
    assert rc == 1 and err.kind == 4


def test_slice16_baseline_matches_oracle(golden):
    """The strong CPU baseline's kernel (slice-by-16 CRC) gives oracle_replay's tuples and errors."""
    assert O.crc32_s16(b"123456789") == 0xCBF43926 == int(golden["crc_check"]["crc32"], 16)
    rng = random.Random(11)
    for n in list(range(0, 40)) + [255, 4096, 65537]:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        assert O.crc32_s16(b) == zlib.crc32(b)
        k = n // 3
        assert O.crc32_s16(b[k:], O.crc32_s16(b[:k])) == zlib.crc32(b)
    for name in ("compaction_example", "persistence"):
        ids, segs = read_dir(name)
        rc, t, err = O.replay(segs)
        rc16, t16, err16 = O.replay_s16(segs)
        assert rc == rc16 == 0 and np.array_equal(t, t16)
    for bad in (bytes.fromhex("0002000000ff00"), b"\x00\x01\x00\x00\x00a\x01", b"\x07\x00\x00\x00\x00"):
        rc, _, err = O.replay([bad])
        rc16, _, err16 = O.replay_s16([bad])
        assert rc == rc16 == 1
        assert (err.kind, err.seg_idx, err.rec_off, err.aux) == (err16.kind, err16.seg_idx, err16.rec_off, err16.aux)


def test_faithful_map_release_is_separate():
    """replay_faithful(release=False) keeps the map (the reference's open() returns it); release frees it."""
    ids, segs = read_dir("compaction_example")
    r1 = O.replay_faithful(segs, release=False)
    O.faithful_release()
    O.faithful_release()   # idempotent
    r2 = O.replay_faithful(segs)
    assert r1[:5] == r2[:5]
