"""KVStore::open bookkeeping on the host (engine.rs:24-28, :59-68), CPU only.

An empty store needs no replay context: kvs_open_ex takes ctx = NULL for a host-only open
(kvstore_host.h), which the C side checks (a store with records returns KVR_EINVAL), so these
tests run without a GPU.  They pin the directory and active-segment behaviour of kvs_open_ex against engine.rs:
  - engine.rs:26-28  fs::create_dir_all(dir) when the directory is missing (nested parents too);
  - engine.rs:59-68  next id = max + 1 (1 for an empty store), segment-<id>.dat created for
                     appends, and a failure to create it is StoreError::Io (KVR_EIO).
"""
import ctypes as C
import os

import pytest

import kvreplay as kv

NO_CTX = None   # host-only open: no context (kvstore_host.h kvs_open_ex)


def open_ex(path, flags=kv.OPEN_HOST_FOLD):
    _, host = kv.native()
    h = C.c_void_p()
    err = kv.Error()
    msg = C.create_string_buffer(4096)
    rc = host.kvs_open_ex(str(path).encode(), NO_CTX, flags, C.byref(h), C.byref(err), msg, len(msg))
    return rc, h


def close(h):
    _, host = kv.native()
    if h.value:
        host.kvs_close(h)


def test_open_creates_nested_directories(tmp_path):
    d = tmp_path / "a" / "b" / "c" / "store"
    rc, h = open_ex(d)
    try:
        assert rc == kv.OK
        assert d.is_dir()
        assert sorted(os.listdir(d)) == ["segment-1.dat"]   # engine.rs:60-68: empty store -> id 1
        assert (d / "segment-1.dat").stat().st_size == 0
        s = kv.StoreStats()
        kv.native()[1].kvs_stats_get(h, C.byref(s))
        assert (s.num_keys, s.total_bytes, s.active_segment_id) == (0, 0, 1)
    finally:
        close(h)


def test_open_existing_directory_next_id(tmp_path):
    d = tmp_path / "store"
    d.mkdir()
    for i in (3, 7):   # empty segments (one per earlier reopen) replay to nothing
        (d / f"segment-{i}.dat").write_bytes(b"")
    # empty segments do need a context for the (trivial) replay: only check discovery here
    assert [i for i, _ in kv.discover(str(d))] == [3, 7]


def test_open_fails_when_the_directory_cannot_be_created(tmp_path):
    f = tmp_path / "file"
    f.write_bytes(b"x")
    rc, h = open_ex(f / "store")   # a parent is a regular file: create_dir_all fails
    close(h)
    assert rc == kv.EIO
    rc, h = open_ex("/proc/self/kvreplay-no-such-dir/store")   # read-only /proc, even for root
    close(h)
    assert rc == kv.EIO


def test_open_fails_when_the_active_segment_cannot_be_created():
    # /proc/self lists no segment-*.dat and refuses new files even for root:
    # engine.rs:62-67 maps the create error to StoreError::Io
    rc, h = open_ex("/proc/self")
    close(h)
    assert rc == kv.EIO


def test_open_fails_when_the_directory_path_is_a_file(tmp_path):
    f = tmp_path / "plain"
    f.write_bytes(b"")
    rc, h = open_ex(f)
    close(h)
    assert rc == kv.EIO


def test_open_without_context_refuses_records(tmp_path):
    d = tmp_path / "store"
    d.mkdir()
    (d / "segment-1.dat").write_bytes(b"")   # empty segments replay to nothing: host-only open works
    rc, h = open_ex(d, 0)
    close(h)
    assert rc == kv.OK
    (d / "segment-2.dat").write_bytes(bytes([1, 1, 0, 0, 0]) + b"k")   # a DEL record: needs the device
    rc, h = open_ex(d, 0)
    close(h)
    assert rc == kv.EINVAL
