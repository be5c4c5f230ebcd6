"""The host-memory transport's join (shadow-1_amd/host/shd_xhost.c, the
engine group's shd_comm of kind "host"), on the CPU: the file compiled on its
own, ranks as forked processes.

A segment left by a group whose rank 0 died still reads ready and can hold a
leftover barrier arrival.  A joiner that finds it must not pass the open
barrier on it (before round 5 the leftover count let it through without any
rank 0, and it failed only at the next collective): it posts a token of its
own and waits for a live rank 0 to echo it; the new rank 0 marks the stale
segment superseded, and the joiner opens the name again and meets it there."""
import ctypes as C
import multiprocessing as mp
import os
import subprocess
import time
import uuid

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def xlib(tmp_path_factory):
    d = tmp_path_factory.mktemp("xh")
    so = str(d / "libxh.so")
    # the transport's functions are hidden in libshdgpu: exported here by wrappers
    src = d / "xh.c"
    src.write_text('#include "%s"\n'
                   '__attribute__((visibility("default"))) int xh_open(const char* n, int w, int r, size_t b, '
                   'shd_xhost** o) { return shd_xhost_open(n, w, r, b, o); }\n'
                   '__attribute__((visibility("default"))) int xh_barrier(shd_xhost* x) '
                   '{ return shd_xhost_barrier(x); }\n'
                   '__attribute__((visibility("default"))) int xh_allgather(shd_xhost* x, const void* m, size_t b, '
                   'void* o) { return shd_xhost_allgather(x, m, b, o); }\n'
                   '__attribute__((visibility("default"))) void xh_close(shd_xhost* x) { shd_xhost_close(x); }\n'
                   % os.path.join(REPO, "shadow-1_amd", "host", "shd_xhost.c"))
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-std=gnu11", "-I", os.path.join(REPO, "include"),
                    "-I", os.path.join(REPO, "shadow-1_amd", "host"), str(src), "-o", so, "-lrt"], check=True)
    return so


def _lib(so):
    lib = C.CDLL(so)
    lib.xh_open.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]
    lib.xh_barrier.argtypes = [C.c_void_p]
    lib.xh_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    lib.xh_close.argtypes = [C.c_void_p]
    return lib


def _stale(so, name, q):
    """a group of two that opens, then rank 1 enters a barrier and both die"""
    def r0():
        lib = _lib(so)
        x = C.c_void_p()
        assert lib.xh_open(name.encode(), 2, 0, 64, C.byref(x)) == 0
        time.sleep(0.5)
        os._exit(0)   # dies without closing: the segment stays, marked ready

    def r1():
        lib = _lib(so)
        x = C.c_void_p()
        assert lib.xh_open(name.encode(), 2, 1, 64, C.byref(x)) == 0
        import threading
        threading.Thread(target=lib.xh_barrier, args=(x,), daemon=True).start()
        time.sleep(0.3)   # arrived (count 1), waiting: dies there, the segment not broken
        os._exit(0)
    ps = [mp.get_context("fork").Process(target=f) for f in (r0, r1)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(20)


def _member(so, name, rank, delay, q):
    lib = _lib(so)
    time.sleep(delay)
    x = C.c_void_p()
    rc = lib.xh_open(name.encode(), 2, rank, 64, C.byref(x))
    if rc:
        q.put((rank, "open", rc))
        return
    mine = C.c_uint64(1000 + rank)
    out = (C.c_uint64 * 2)()
    rc = lib.xh_allgather(x, C.byref(mine), 8, out)
    q.put((rank, "gather", rc, list(out)))
    lib.xh_close(x)


def test_joiner_does_not_pass_a_stale_segment(xlib):
    name = "shdxh_" + uuid.uuid4().hex[:12]
    os.environ["SHD_XHOST_TIMEOUT"] = "20"
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    st = ctx.Process(target=_stale, args=(xlib, name, q))
    st.start()
    st.join(30)
    assert os.path.exists("/dev/shm/" + name)   # the stale segment is there
    # the joiner first (it finds the stale segment), the new rank 0 a second later
    ps = [ctx.Process(target=_member, args=(xlib, name, 1, 0.0, q)),
          ctx.Process(target=_member, args=(xlib, name, 0, 1.0, q))]
    for p in ps:
        p.start()
    res = [q.get(timeout=60) for _ in range(2)]
    for p in ps:
        p.join(30)
    try:
        os.unlink("/dev/shm/" + name)
    except OSError:
        pass
    assert sorted(r[:3] for r in res) == [(0, "gather", 0), (1, "gather", 0)], res
    assert all(r[3] == [1000, 1001] for r in res)
