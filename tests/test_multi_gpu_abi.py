"""kvr_replay_multi (include/kvreplay.h) through the C ABI: segments dealt round-robin
over several contexts, each shard replayed on its own host thread, merged on the host.  Every test
runs on repeated device 0 (contexts on one GPU stand in for GPUs) and, on a box with enough GPUs,
on distinct devices (per-thread hipSetDevice, one stream per device).  The result must be bit-exact with the oracle's replay
of the whole store: every tuple field in (segment, offset) order, the manifest verification flags,
and the store's first error (the minimum (segment, offset) over the shards, engine.rs:56)."""
import glob
import os

import numpy as np
import pytest

import kvreplay as K
import oracle_py as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SPEC = K.GenSpec(seed=0x3C7A, seg_bytes=300_000, val_min=16, val_max=5000, del_permille=300,
                 key_space_log2=10, flip_per_million=3000)


def _n_gpus():
    """GPUs this process may use, from the KFD topology (no HIP call): the GPU nodes, or as many as
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES name."""
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(f) as fh:
                props = dict(line.split() for line in fh if len(line.split()) == 2)
            n += int(props.get("simd_count", "0")) > 0
        except (OSError, ValueError):
            pass
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def device_lists(n):
    """[0] * n always; [0, 1, .., n-1] too (skipped at run time, not collection, on a box with fewer
    GPUs: see _enough_gpus)."""
    return [pytest.param([0] * n, id=f"dev0x{n}"), pytest.param(list(range(n)), id=f"dev{n}")]


@pytest.fixture(autouse=True)
def _enough_gpus(request):
    cs = getattr(request.node, "callspec", None)
    devs = cs.params.get("devices") if cs is not None else None
    if devs and len(set(devs)) > 1 and _n_gpus() < len(set(devs)):
        pytest.skip(f"needs {len(set(devs))} GPUs")


def _store(n):
    parts = [K.gen_segment_cpu(SPEC, s) for s in range(n)]
    return [p[0].tobytes() for p in parts], np.concatenate([p[1] for p in parts])


@pytest.mark.parametrize("n_segs", [5, 1, 7, 2])
@pytest.mark.parametrize("devices", device_lists(2) + device_lists(3))
def test_multi_matches_oracle(devices, n_segs):
    segs, man = _store(n_segs)
    mc = K.MultiContext(devices)
    try:
        ids = [10 + 3 * i for i in range(n_segs)]
        r = mc.replay(segs, seg_ids=ids)
        rc, ref, _ = O.replay(segs, seg_ids=ids)
        assert r.status == rc == 0 and np.array_equal(r.tuples, ref)
        assert r.stats.n_shards == len(devices) and r.stats.n_records == len(ref)
        # the manifest in store order: flips injected by the generator fail, everything else passes
        r = mc.replay(segs, expected=man)
        rc, ref, _ = O.replay(segs, expected=man)
        assert r.status == rc == 0 and np.array_equal(r.tuples, ref)
        fails = int(np.count_nonzero(ref["flags"] & K.TF_CRC_FAIL))
        assert r.stats.n_crc_fail == fails and (fails > 0 or n_segs < 5)
    finally:
        mc.close()


@pytest.mark.parametrize("devices", device_lists(2))
def test_multi_first_error_is_store_minimum(devices):
    segs, _ = _store(6)
    bad = list(segs)
    bad[4] = bad[4][:-3]           # shard 0 (segments 0, 2, 4): torn tail
    bad[3] = bad[3][:-1]           # shard 1 (segments 1, 3, 5): torn earlier in the store
    bad[5] = b"\x07" + bad[5][1:]  # a bad opcode after both
    mc = K.MultiContext(devices)
    try:
        r = mc.replay(bad)
        rc, _, e = O.replay(bad)
        assert r.status == rc == K.CORRUPTED
        assert (r.error.kind, r.error.seg_idx, r.error.rec_off, r.error.aux) == (e.kind, e.seg_idx, e.rec_off, e.aux)
        assert r.error.seg_idx == 3
    finally:
        mc.close()


@pytest.mark.parametrize("devices", device_lists(2))
def test_multi_empty_and_capacity(devices):
    mc = K.MultiContext(devices)
    try:
        r = mc.replay([])
        assert r.status == 0 and r.n == 0
        segs, _ = _store(3)
        r = mc.replay([b""] + segs + [b""], cap=5)     # too small: the wrapper retries with the exact count
        rc, ref, _ = O.replay([b""] + segs + [b""])
        assert r.status == rc == 0 and np.array_equal(r.tuples, ref)
    finally:
        mc.close()


@pytest.mark.parametrize("devices", device_lists(2) + device_lists(3))
def test_live_multi_matches_oracle_fold(devices):
    """kvr_replay_live_multi: per-GPU reduction to every key's last record (tombstones kept: a DEL
    in one shard deletes a key SET in another), host merge by (segment, offset) -> exactly the
    oracle's live map of the whole store."""
    spec = K.GenSpec(seed=104, seg_bytes=400_000, key_space_log2=9, val_min=0, val_max=200, del_permille=350)
    segs = [K.gen_segment_cpu(spec, s)[0] for s in range(7)]
    ids = [2, 3, 5, 8, 13, 21, 34]
    rc, t, _ = O.replay(segs, seg_ids=ids)
    live, nk, tb = O.fold_live(segs, t)
    m = K.MultiContext(devices)
    try:
        r = m.replay(segs, seg_ids=ids, live=True)
        assert r.status == 0 and r.n == nk and np.array_equal(r.tuples, t[live])
        bad = segs[:4] + [segs[4][:-3]] + segs[5:]
        rc2, _, err = O.replay(bad, seg_ids=ids)
        r = m.replay(bad, seg_ids=ids, live=True)
        assert r.status == 1 and (r.error.kind, r.error.seg_idx, r.error.rec_off) == (err.kind, err.seg_idx, err.rec_off)
    finally:
        m.close()


@pytest.mark.parametrize("devices", device_lists(2) + device_lists(3))
def test_live_multi_device_resident_with_keys(devices):
    """The sharded index of a store that lives in HBM (BASELINE cfg4/cfg5 shape: generated on the
    device, never on the host): kvr_replay_live_multi with KVR_SEGS_ON_DEVICE, segment i on
    context i mod N.  Keys repeat across segments and 35 % of records are DELs, so tombstones cross
    shards.  The live tuples equal the oracle's fold of the whole store (engine.rs:137 / :141) and
    the exported key bytes (kvr_multi_live_keys) equal the oracle's keys of those records.
    Segment i is generated on, and stays in the HBM of, device devices[i mod N]."""
    spec = K.GenSpec(seed=108, seg_bytes=250_000, key_space_log2=9, val_min=0, val_max=300, del_permille=350)
    n = 7
    ids = [1, 4, 9, 16, 25, 36, 49]
    host = [K.gen_segment_cpu(spec, s)[0] for s in range(n)]   # byte-identical to the device generator
    rc, t, _ = O.replay(host, seg_ids=ids)
    live, nk, _ = O.fold_live(host, t)
    want = t[live]
    wkeys = [bytes(host[x["seg_idx"]][x["rec_off"] + 5: x["rec_off"] + 5 + x["key_len"]]) for x in want]
    nd = len(devices)
    gens = {d: K.Context(d) for d in sorted(set(devices))}
    m = K.MultiContext(devices)
    try:
        sizes = [len(h) for h in host]
        bufs = {d: torch.zeros(sum(s + 256 for s in sizes) + 256, dtype=torch.uint8, device=f"cuda:{d}")
                for d in gens}
        offs = {d: 16 for d in gens}
        ptrs = []
        for s, ln in enumerate(sizes):
            d = devices[s % nd]
            p = bufs[d].data_ptr() + offs[d]
            got = gens[d].gen_segment_device(spec, s, p, ln)
            assert got[0] == ln
            ptrs.append((p, ln))
            offs[d] += ln + 256 + (s % 5)          # odd device alignments
        for d in gens:
            torch.cuda.synchronize(d)
        r = m.replay(ptrs, seg_ids=ids, live=True, on_device=True)
        assert r.status == 0 and r.n == nk and np.array_equal(r.tuples, want)
        keys, offs = m.live_keys(r.n)
        assert offs[0] == 0 and int(offs[-1]) == len(keys)
        assert [bytes(keys[offs[i]: offs[i + 1]]) for i in range(r.n)] == wkeys
        # the plain (all tuples) multi replay from device shards too
        r2 = m.replay(ptrs, seg_ids=ids, on_device=True)
        assert r2.status == 0 and np.array_equal(r2.tuples, t)
        # a torn device segment: the store's first error, as from host bytes
        bad = list(ptrs)
        bad[4] = (ptrs[4][0], ptrs[4][1] - 3)
        rcb, _, err = O.replay(host[:4] + [host[4][:-3]] + host[5:], seg_ids=ids)
        r3 = m.replay(bad, seg_ids=ids, live=True, on_device=True)
        assert r3.status == rcb == 1
        assert (r3.error.kind, r3.error.seg_idx, r3.error.rec_off) == (err.kind, err.seg_idx, err.rec_off)
    finally:
        m.close()
        for g in gens.values():
            g.close()


@pytest.mark.parametrize("devices", device_lists(8))
def test_eight_way_cfg4_shape(devices):
    """The target width (BASELINE cfg4: segments dealt round-robin over 8 GPUs, 50 % tombstones):
    16 segments over 8 contexts, so each shard holds two segments and a key SET in one shard is
    deleted in others.  kvr_replay_live_multi equals the oracle's fold of the whole store
    (engine.rs:137 / :141), kvr_replay_multi its tuples, and the store's first error is the
    minimum (segment, offset) over the shards (engine.rs:56)."""
    spec = K.GenSpec(seed=0xC4F8, seg_bytes=200_000, key_space_log2=10, val_min=0, val_max=1024, del_permille=500)
    n = 16
    ids = [3 * i + 1 for i in range(n)]
    segs = [K.gen_segment_cpu(spec, s)[0].tobytes() for s in range(n)]
    rc, t, _ = O.replay(segs, seg_ids=ids)
    live, nk, tb = O.fold_live(segs, t)
    assert rc == 0 and tb > 0
    m = K.MultiContext(devices)
    try:
        r = m.replay(segs, seg_ids=ids, live=True)
        assert r.status == 0 and r.n == nk and np.array_equal(r.tuples, t[live])
        assert r.stats.n_shards == 8
        r = m.replay(segs, seg_ids=ids)
        assert r.status == 0 and np.array_equal(r.tuples, t)
        bad = list(segs)
        bad[13] = bad[13][:-2]     # shard 5
        bad[6] = bad[6][:-1]       # shard 6, earlier in the store: the store's error
        rcb, _, err = O.replay(bad, seg_ids=ids)
        r = m.replay(bad, seg_ids=ids, live=True)
        assert r.status == rcb == K.CORRUPTED and err.seg_idx == 6
        assert (r.error.kind, r.error.seg_idx, r.error.rec_off, r.error.aux) == (err.kind, err.seg_idx, err.rec_off, err.aux)
    finally:
        m.close()
