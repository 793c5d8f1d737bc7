"""CPU-side tests of the product libraries: ABI exports, host logic, generator (no GPU calls)."""
import os
import re
import zlib

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M64 = (1 << 64) - 1


def header_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(kv[a-z]_\w+)\s*\(", src, flags=re.M))


def test_abi_exports_every_declared_function():
    rep_p, host_p = K.lib_paths()
    import subprocess
    def exports(p):
        out = subprocess.run(["nm", "-D", "--defined-only", p], capture_output=True, text=True).stdout
        return {l.split()[-1] for l in out.splitlines() if " T " in l}
    ex = exports(rep_p) | exports(host_p)
    decl = header_functions(os.path.join(ROOT, "include", "kvreplay.h")) | \
        header_functions(os.path.join(ROOT, "include", "kvstore_host.h"))
    assert len(decl) >= 20
    missing = sorted(decl - ex)
    assert not missing, missing
    rep, host = K.native()          # and they load (without a GPU)
    assert rep.kvr_strerror(1) == b"corrupted data"


def test_tuple_layout_is_32_bytes():
    assert K.TUPLE_DTYPE.itemsize == 32
    assert [K.TUPLE_DTYPE.fields[f][1] for f in ("rec_off", "seg_idx", "key_len", "val_len", "crc32", "key_tag",
                                                 "op", "flags")] == [0, 8, 12, 16, 20, 24, 28, 29]


def test_host_crc32_matches_zlib():
    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 16, 100, 4097):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert K.crc32(b) == zlib.crc32(b)


# ---- generator restated in Python (kvr_gen_common.h) -----------------------------------------
def mix64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def py_gen(spec, seg_no):
    sbase = mix64(spec.seed ^ mix64(seg_no ^ 0x5EB5EB5EB5EB5EB5))
    r = lambda i, k: mix64(sbase ^ mix64(((i << 4) | k) & M64))
    out, exp, i = bytearray(), [], 0
    while True:
        op = 1 if r(i, 0) % 1000 < spec.del_permille else 0
        ksl = min(max(spec.key_space_log2, 1), 48)
        if spec.key_dist == 0:
            kid = r(i, 1) & ((1 << ksl) - 1)
        else:
            b = r(i, 1) % ksl
            kid = (1 << b) - 1 + (r(i, 2) & ((1 << b) - 1))
        if op:
            vlen = 0
        elif spec.val_min >= spec.val_max:
            vlen = spec.val_min
        else:
            lo = max(spec.val_min, 1)
            nb = 0
            while nb < 31 and (lo << (nb + 1)) <= spec.val_max:
                nb += 1
            if nb == 0:
                vlen = lo + r(i, 3) % (spec.val_max - lo + 1)
            else:
                o = r(i, 3) % nb
                base = lo << o
                vlen = base + r(i, 4) % base
        size = 21 if op else 25 + vlen
        if len(out) + size > spec.seg_bytes:
            break
        key = b"k" + b"%015d" % (kid % 10 ** 15)
        if op:
            out += b"\x01" + (16).to_bytes(4, "little") + key
            exp.append(0)
        else:
            vs = r(i, 5)
            v = bytearray(b"".join(mix64((vs + j) & M64).to_bytes(8, "little") for j in range((vlen + 7) // 8))[:vlen])
            exp.append(zlib.crc32(bytes(v)))
            if vlen and r(i, 6) % 1000000 < spec.flip_per_million:
                fb = r(i, 7) % (8 * vlen)
                v[fb >> 3] ^= 1 << (fb & 7)
            out += b"\x00" + (16).to_bytes(4, "little") + key + vlen.to_bytes(4, "little") + bytes(v)
        i += 1
    return bytes(out), np.array(exp, dtype=np.uint32)


SPECS = [
    K.GenSpec(seed=1, seg_bytes=20000, val_min=64, val_max=64),
    K.GenSpec(seed=2, seg_bytes=30000, key_dist=1, key_space_log2=24, val_min=16, val_max=4096, del_permille=100),
    K.GenSpec(seed=3, seg_bytes=30000, val_min=1, val_max=700, del_permille=500, flip_per_million=200000),
]


@pytest.mark.parametrize("spec", SPECS)
def test_cpu_generator_matches_python_restatement(spec):
    for seg_no in (0, 5):
        b, e = K.gen_segment_cpu(spec, seg_no)
        pb, pe = py_gen(spec, seg_no)
        assert b.tobytes() == pb
        assert np.array_equal(e, pe)


@pytest.mark.parametrize("spec", SPECS)
def test_generated_segments_replay_and_verify_on_oracle(spec):
    segs, exps = zip(*[K.gen_segment_cpu(spec, s) for s in range(3)])
    exp = np.concatenate(exps)
    rc, t, err = O.replay(list(segs), expected=exp)
    assert rc == 0 and len(t) == len(exp)
    sets = t["op"] == 0
    assert np.all(t["flags"][sets] & K.TF_VERIFIED)
    fails = (t["flags"] & K.TF_CRC_FAIL) != 0
    assert np.array_equal(fails, sets & (t["crc32"] != exp))
    if spec.flip_per_million == 0:
        assert not fails.any()
    else:
        assert fails.any()


def test_native_fold_matches_oracle_fold():
    spec = SPECS[2]
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(4)]
    rc, t, _ = O.replay(segs)
    assert rc == 0
    live_o, nk_o, tb_o = O.fold_live(segs, t)
    live_n, nk_n, tb_n = K.fold(segs, t)
    assert (nk_o, tb_o) == (nk_n, tb_n)
    assert np.array_equal(live_o, live_n)


@pytest.mark.parametrize("threads", [0, 2, 3, 8, 17])
def test_parallel_fold_matches_oracle_fold(threads):
    # keys repeat across segments and partitions (2^10 ids, 40 % DEL, a DEL of an absent key)
    spec = K.GenSpec(seed=99, seg_bytes=120_000, key_space_log2=10, val_min=0, val_max=300, del_permille=400)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(5)]
    segs.append(np.frombuffer(b"\x01\x05\x00\x00\x00nokey", dtype=np.uint8))
    rc, t, _ = O.replay(segs)
    assert rc == 0
    live_o, nk_o, tb_o = O.fold_live(segs, t)
    live_p, nk_p, tb_p = K.fold(segs, t, threads=threads)
    assert (nk_o, tb_o) == (nk_p, tb_p)
    assert np.array_equal(live_o, live_p)
    assert K.fold([], t[:0], threads=threads)[1:] == (0, 0)


@pytest.mark.parametrize("s,v", [("0", 0), ("001", 1), ("+7", 7), ("18446744073709551615", 2 ** 64 - 1),
                                 ("18446744073709551616", None), ("", None), ("+", None), ("-1", None),
                                 (" 1", None), ("1a", None), ("++1", None)])
def test_rust_u64_parse(s, v):
    assert K.parse_u64(s) == v


def test_discover_follows_engine_rs(tmp_path):
    names = ["segment-10.dat", "segment-2.dat", "segment-+3.dat", "segment-007.dat", "segment-.dat",
             "segment-x.dat", "segment-1.dat.bak", "notes.txt", "segment-18446744073709551616.dat"]
    for n in names:
        (tmp_path / n).write_bytes(b"")
    got = K.discover(str(tmp_path))
    assert [i for i, _ in got] == [2, 3, 7, 10]
    assert [os.path.basename(p) for _, p in got] == ["segment-2.dat", "segment-+3.dat", "segment-007.dat",
                                                     "segment-10.dat"]


def test_format_error_messages():
    p = "db/segment-1.dat"
    assert K.format_error(2, 0, 5, 0, p) == "Failed to read key length in db/segment-1.dat: failed to fill whole buffer"
    assert K.format_error(3, 0, 5, 0, p) == "Failed to read key in db/segment-1.dat: failed to fill whole buffer"
    assert K.format_error(4, 0, 0, (1 << 32) | 2, p) == \
        "Invalid UTF-8 key in db/segment-1.dat: invalid utf-8 sequence of 1 bytes from index 2"
    assert K.format_error(4, 0, 0, 3, p) == "Invalid UTF-8 key in db/segment-1.dat: incomplete utf-8 byte sequence from index 3"
    assert K.format_error(5, 0, 0, 0, p) == "Failed to read val len in db/segment-1.dat: failed to fill whole buffer"
    assert K.format_error(6, 0, 0, 0, p) == "Failed to read val in db/segment-1.dat: failed to fill whole buffer"
    assert K.format_error(7, 0, 0, 9, p) == "Unknown opcode 9 in segment db/segment-1.dat"


def test_segment_list_marshals_like_a_list():
    """kvreplay.SegmentList (the kvr_segment array marshaled once, bench.py's replay step) holds
    the same ids, pointers and lengths Context.replay builds from a plain list."""
    segs = [b"\x00\x01\x00\x00\x00k\x01\x00\x00\x00v", bytearray(b""), np.arange(7, dtype=np.uint8)]
    sl = K.SegmentList(segs, seg_ids=[3, 5, 9])
    assert len(sl) == 3 and sl.total == 11 + 0 + 7 and not sl.on_device
    assert [sl.arr[i].seg_id for i in range(3)] == [3, 5, 9]
    assert [sl.arr[i].len for i in range(3)] == [11, 0, 7]
    assert sl.arr[0].bytes == sl.keep[0].ctypes.data and not sl.arr[1].bytes
    dev = K.SegmentList([(0x1000, 64), (0x2000, 0)], on_device=True)
    assert dev.on_device and [dev.arr[i].seg_id for i in range(2)] == [0, 1]
    assert [(dev.arr[i].bytes, dev.arr[i].len) for i in range(2)] == [(0x1000, 64), (0x2000, 0)]
