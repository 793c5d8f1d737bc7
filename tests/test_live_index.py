"""GPU parity of kvr_replay_live (replay + last-writer fold in HBM, SURVEY §8b dedup_last_writer).

The output must be exactly the oracle's tuples whose record is its key's final SET
(engine.rs:137 insert / :141 remove, in (segment, offset) order): the records the reference's
HashMap holds after KVStore::open.  Its count is stats().num_keys.
"""
import os

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _expect(segs, seg_ids=None):
    rc, t, err = O.replay(segs, seg_ids=seg_ids)
    if rc != 0:
        return rc, None, err
    live, nk, tb = O.fold_live(segs, t)
    return rc, t[live], (nk, tb)


def _check(ctx, segs, seg_ids=None):
    rc, want, extra = _expect(segs, seg_ids)
    r = ctx.replay_live(segs, seg_ids=seg_ids)
    assert r.status == rc
    if rc == 0:
        assert r.n == len(want) == extra[0]
        assert np.array_equal(r.tuples, want)
        assert int(r.tuples["val_len"].astype(np.uint64).sum()) == extra[1]   # stats().total_bytes
    else:
        assert (r.error.kind, r.error.seg_idx, r.error.rec_off) == (extra.kind, extra.seg_idx, extra.rec_off)
    return r


@pytest.mark.parametrize("name", ["persistence", "store_integration", "compaction_example", "large_dataset"])
def test_live_index_golden(gctx, name):
    d = os.path.join(GOLD, name)
    names = sorted((n for n in os.listdir(d) if n.startswith("segment-")), key=lambda n: int(n[8:-4]))
    segs = [open(os.path.join(d, n), "rb").read() for n in names]
    _check(gctx, segs, seg_ids=[int(n[8:-4]) for n in names])


@pytest.mark.parametrize("spec", [
    K.GenSpec(seed=91, seg_bytes=400_000, key_space_log2=10, val_min=0, val_max=300, del_permille=400),
    K.GenSpec(seed=92, seg_bytes=700_000, val_min=1024, val_max=1024, del_permille=500),
    K.GenSpec(seed=93, seg_bytes=2_000_000, key_dist=1, key_space_log2=24, val_min=16, val_max=1 << 20,
              del_permille=100),
])
def test_live_index_generated(gctx, spec):
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(5)]
    _check(gctx, segs)


def test_live_index_error_and_capacity(gctx):
    spec = K.GenSpec(seed=94, seg_bytes=200_000, key_space_log2=8, val_min=0, val_max=64, del_permille=300)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(3)]
    _check(gctx, segs[:1] + [segs[1][:-2]] + segs[2:])      # first error, as kvr_replay reports it
    rc, want, _ = _expect(segs)
    r = gctx.replay_live(segs, cap=3)                           # KVR_CAPACITY, then the retry
    assert r.status == 0 and np.array_equal(r.tuples, want)
    assert gctx.replay_live([]).n == 0
