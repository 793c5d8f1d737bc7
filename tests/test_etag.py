"""Batch ETag compute / verify (kvr_etag_batch) against zlib.crc32.

The ETag is format!("{:08x}", crc32fast::hash(data)) (src/volume/storage.rs:27): CRC-32/ISO-HDLC,
which Python's zlib.crc32 implements identically (check value "123456789" -> cbf43926).
"""
import json
import os
import random
import zlib

import numpy as np
import pytest

import kvreplay as K

HERE = os.path.dirname(os.path.abspath(__file__))


def test_etag_format_cpu():
    assert K.etag_format(0xCBF43926) == "cbf43926"
    assert K.etag_format(0) == "00000000"
    assert K.etag_format(0x0000ABCD) == "0000abcd"


@pytest.mark.gpu
def test_etag_check_value_and_golden_values(gctx):
    blobs = [b"123456789", b"", b"first", b"42", b"Test Store", b"43"]
    data = b"".join(blobs)
    offs = np.cumsum([0] + [len(b) for b in blobs[:-1]])
    crc, nf, _ = gctx.etag_batch(data, offs, [len(b) for b in blobs])
    assert K.etag_format(int(crc[0])) == "cbf43926"
    assert [int(c) for c in crc] == [zlib.crc32(b) for b in blobs]
    # the persistence example's values: session, counter, name; counter after seg 2
    assert [K.etag_format(int(c)) for c in crc[2:]] == ["9271ee57", "3224b088", "80616dbc", "4523801e"]


# lengths around the 64-B lane unit and the 4-KiB chunk, multi-chunk blobs past one wave's 64
# chunks, at every alignment
LENS = [0, 1, 3, 4, 5, 63, 64, 65, 127, 4095, 4096, 4097, 8191, 65536, 65536 + 7, 64 * 4096, 64 * 4096 + 1,
        65 * 4096 + 13, 130 * 4096 - 1, (1 << 20) + 5]


@pytest.mark.gpu
@pytest.mark.parametrize("on_device", [False, True])
def test_etag_matches_zlib(gctx, on_device):
    rng = random.Random(7)
    offs, lens, pos = [], [], 0
    for ln in LENS * 2:
        pos += rng.randrange(0, 16)          # unaligned starts
        offs.append(pos)
        lens.append(ln)
        pos += ln
    data = np.frombuffer(rng.randbytes(pos + 1), dtype=np.uint8)[: pos]   # last blob ends at the buffer end
    offs += [0, 5, pos - 3]                  # overlapping blobs, a tail blob
    lens += [pos, 4096 * 3, 3]
    exp = [zlib.crc32(data[o:o + n].tobytes()) for o, n in zip(offs, lens)]
    if on_device:
        torch = pytest.importorskip("torch")
        d = torch.from_numpy(data.copy()).to("cuda:0")
        torch.cuda.synchronize()
        crc, nf, st = gctx.etag_batch(d.data_ptr(), offs, lens, on_device=True, data_len=len(data))
    else:
        crc, nf, st = gctx.etag_batch(data, offs, lens)
    assert [int(c) for c in crc] == exp
    assert st.bytes == sum(lens) and st.n_blobs == len(lens)


@pytest.mark.gpu
def test_etag_verify_counts_mismatches(gctx):
    rng = np.random.default_rng(3)
    n, size = 3000, 2000
    data = rng.integers(0, 256, n * size, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * size
    lens = np.full(n, size, dtype=np.uint64)
    exp = np.array([zlib.crc32(data[i * size:(i + 1) * size].tobytes()) for i in range(n)], dtype=np.uint32)
    bad = rng.choice(n, 17, replace=False)
    stored = exp.copy()
    stored[bad] ^= 1 << 5                    # stale ETags: the scrub must flag exactly these
    crc, nf, _ = gctx.etag_batch(data, offs, lens, expected=stored)
    assert np.array_equal(crc, exp)
    assert nf == 17


@pytest.mark.gpu
def test_etag_rejects_blob_outside_buffer(gctx):
    with pytest.raises(K.NativeError):
        gctx.etag_batch(b"abc", [1], [3])
    crc, nf, _ = gctx.etag_batch(b"", [], [])
    assert len(crc) == 0 and nf == 0
