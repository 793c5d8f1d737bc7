"""Generate the committed golden fixtures (run: python tests/golden/make_golden.py).

The segment files are produced by restating the reference writer's framing exactly
(src/store/engine.rs:157-198):
    set:    [0u8][key_len u32 LE][key][val_len u32 LE][value]   engine.rs:169-173
    delete: [1u8][key_len u32 LE][key]                           engine.rs:191-193
replaying the write sequences of the reference's own tests/examples:
    persistence/        examples/persistence.rs:7-13 (session 1 -> segment-1.dat),
                        :41-48 (session 2 -> segment-2.dat), :53 (session 3 open -> empty segment-3.dat)
    store_integration/  tests/store_integration.rs:12-18 (5 rounds x 100 keys, one segment)
    compaction_example/ examples/compaction.rs:10-15 (10 rounds x 100 keys)
    large_dataset/      examples/large_dataset.rs:14-17 (10,000 keys)
Every KVStore::open of a fresh directory writes into segment-1.dat (engine.rs:60-62: max id 0 + 1).

golden.json pins what the reference's asserts state (final maps / key counts) plus the derived
tuple constants of SURVEY.md §8c, the file sizes and zlib CRC-32s, and a set of negative cases
whose expected CorruptedData kind follows the check order of engine.rs:85-149.
"""
import json
import os
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))


def rec_set(k: bytes, v: bytes) -> bytes:
    return b"\x00" + len(k).to_bytes(4, "little") + k + len(v).to_bytes(4, "little") + v


def rec_del(k: bytes) -> bytes:
    return b"\x01" + len(k).to_bytes(4, "little") + k


def write(dirname, files):
    d = os.path.join(HERE, dirname)
    os.makedirs(d, exist_ok=True)
    for name, data in files.items():
        with open(os.path.join(d, name), "wb") as f:
            f.write(data)
    return {name: {"size": len(data), "crc32": "%08x" % zlib.crc32(data)} for name, data in files.items()}


def main():
    out = {"crc_check": {"input": "123456789", "crc32": "%08x" % zlib.crc32(b"123456789")}}

    # examples/persistence.rs
    s1 = rec_set(b"session", b"first") + rec_set(b"counter", b"42") + rec_set(b"name", b"Test Store")
    s2 = rec_set(b"counter", b"43") + rec_del(b"name")
    out["persistence"] = {
        "files": write("persistence", {"segment-1.dat": s1, "segment-2.dat": s2, "segment-3.dat": b""}),
        "hex_segment_1": s1.hex(),
        "hex_segment_2": s2.hex(),
        # session 2 replays segment-1 only (persistence.rs:17-37): (key, seg_id, rec_off, val_off, vlen, crc)
        "after_segment_1": [["session", 1, 0, 16, 5, "9271ee57"], ["counter", 1, 21, 37, 2, "3224b088"],
                            ["name", 1, 39, 52, 10, "80616dbc"]],
        "after_segment_1_stats": {"num_keys": 3, "total_bytes": 17},
        # session 3 (persistence.rs:53-67): counter updated, name deleted (DEL at (2, 18))
        "after_all": [["session", 1, 0, 16, 5, "9271ee57"], ["counter", 2, 0, 16, 2, "4523801e"]],
        "after_all_stats": {"num_keys": 2, "total_bytes": 7},
        "values_after_all": {"session": "first", "counter": "43"},
        "absent_after_all": ["name"],
    }

    # tests/store_integration.rs:12-18
    si = b"".join(rec_set(b"key_%d" % i, b"value_%d_%d" % (i, r)) for r in range(5) for i in range(100))
    out["store_integration"] = {
        "files": write("store_integration", {"segment-1.dat": si}),
        "rounds": 5, "keys": 100, "num_keys": 100, "total_bytes": 990,
        "key_0": {"rec_off": 9920, "val_off": 9934, "vlen": 9, "crc32": "%08x" % zlib.crc32(b"value_0_4")},
        "key_99": {"rec_off": 12375, "val_off": 12390, "vlen": 10},
    }

    # examples/compaction.rs:10-15
    ce = b"".join(rec_set(b"key_%d" % i, b"value_%d_%d" % (i, r)) for r in range(10) for i in range(100))
    out["compaction_example"] = {
        "files": write("compaction_example", {"segment-1.dat": ce}),
        "rounds": 10, "keys": 100, "num_keys": 100, "total_bytes": 990,
    }

    # examples/large_dataset.rs:14-17
    ld = b"".join(rec_set(b"user:%05d:data" % i, b"User data for ID %d" % i) for i in range(10000))
    out["large_dataset"] = {
        "files": write("large_dataset", {"segment-1.dat": ld}),
        "num_keys": 10000, "total_bytes": 208890,
        "samples": {"user:00000:data": "User data for ID 0", "user:09999:data": "User data for ID 9999",
                    "user:05000:data": "User data for ID 5000"},
    }

    # Negative cases (engine.rs:85-149).  kind names as in kvreplay.h; off = failing record offset.
    good = rec_set(b"alpha", b"one") + rec_del(b"beta")          # 22 + 10 = 32 bytes
    neg = []

    def case(name, data, kind, off, aux=None):
        neg.append({"name": name, "hex": data.hex(), "kind": kind, "off": off, "aux": aux})

    case("empty_segment", b"", "NONE", None)
    case("exact_boundary", good, "NONE", None)
    for cut in range(1, 5):
        case(f"tail_op_plus_{cut - 1}_len_bytes", good + rec_set(b"k", b"v")[:cut], "KEY_LEN", len(good))
    case("tail_short_key", good + rec_set(b"key", b"v")[:7], "KEY", len(good))
    case("tail_no_vlen", good + rec_set(b"key", b"v")[:8 + 2], "VAL_LEN", len(good))
    case("tail_short_val", good + rec_set(b"key", b"value")[:-2], "VAL", len(good))
    case("huge_key_len", good + b"\x00\xff\xff\xff\xff" + b"abc", "KEY", len(good))
    case("opcode_2", good + b"\x02" + (3).to_bytes(4, "little") + b"xyz", "OPCODE", len(good), 2)
    case("opcode_255_empty_key", b"\xff" + bytes(4), "OPCODE", 0, 255)
    case("opcode_after_bad_utf8", b"\x07" + (2).to_bytes(4, "little") + b"\xc3\x28", "UTF8", 0, [0, 1])
    case("bad_utf8_ff", good + rec_set(b"ab\xffcd", b"v"), "UTF8", len(good), [2, 1])
    case("bad_utf8_incomplete", rec_set(b"ok", b"1") + rec_del(b"x\xe2\x82"), "UTF8", len(rec_set(b"ok", b"1")), [1, 0])
    case("bad_utf8_surrogate", rec_set(b"\xed\xa0\x80", b"v"), "UTF8", 0, [0, 1])
    case("bad_utf8_overlong", rec_set(b"a\xc0\xafb", b"v"), "UTF8", 0, [1, 1])
    case("bad_utf8_3byte_2nd", rec_set(b"\xe2\x82\x28", b"v"), "UTF8", 0, [0, 2])
    case("bad_utf8_4byte_3rd", rec_set(b"\xf0\x9f\x98\x28", b"v"), "UTF8", 0, [0, 3])
    case("valid_utf8_multibyte", rec_set("é€😀".encode(), b"v") + rec_del("ключ".encode()), "NONE", None)
    case("delete_absent_key", rec_del(b"ghost") + rec_set(b"a", b"b"), "NONE", None)
    case("empty_key_and_value", rec_set(b"", b"") + rec_set(b"", b"x") + rec_del(b""), "NONE", None)
    out["negative"] = neg

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
