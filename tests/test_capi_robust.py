"""C ABI robustness (no GPU needed): malformed calls — NULL pointers, orders
outside 1..64, unknown dtype / kernel / schedule codes, bad thread counts,
too-small output buffers — return a negative SUP_E* code with a message and
never crash the caller ("never exit()").  Each group runs in a
child process, so a crash fails the test instead of the test runner."""
import os
import subprocess
import sys
import textwrap

from conftest import ROOT

CHILD = textwrap.dedent(r"""
    import ctypes as C, sys
    sys.path.insert(0, ROOT)
    import numpy as np
    from superman_amd import _lib
    lib = _lib.load()
    lib.sup_last_error.restype = C.c_char_p
    a = np.ones((6, 6), dtype=np.float64)
    big = np.ones((65, 65), dtype=np.float64)
    out, st = C.c_double(0.0), _lib.SupStats()
    o = _lib.SupOpts() if hasattr(_lib, "SupOpts") else None
    P = a.ctypes.data
    codes = {}

    def call(name, *args):
        rc = getattr(lib, name)(*args)
        codes[name + repr(len(codes))] = rc
        msg = lib.sup_last_error()
        assert rc < 0, (name, rc)
        assert msg, (name, "no message")

    # sup_perman_cpu: host walk entry point (validates before computing)
    call("sup_perman_cpu", None, 0, 6, 0, 4, C.byref(out), C.byref(st))
    call("sup_perman_cpu", C.c_void_p(P), 0, 0, 0, 4, C.byref(out), C.byref(st))
    call("sup_perman_cpu", C.c_void_p(P), 0, -3, 0, 4, C.byref(out), C.byref(st))
    call("sup_perman_cpu", C.c_void_p(big.ctypes.data), 0, 65, 0, 4, C.byref(out), C.byref(st))
    call("sup_perman_cpu", C.c_void_p(P), 77, 6, 0, 4, C.byref(out), C.byref(st))
    call("sup_perman_cpu", C.c_void_p(P), 0, 6, 99, 4, C.byref(out), C.byref(st))
    call("sup_perman_cpu", C.c_void_p(P), 0, 6, 0, 4, None, C.byref(st))
    # sup_perman / sup_partial / sup_perman_shard (GPU entry points: the
    # arguments are checked before any device is touched, or the device check fails)
    call("sup_perman", None, 0, 6, 0, 0, None, C.byref(out), None)
    call("sup_perman", C.c_void_p(P), 0, 0, 0, 0, None, C.byref(out), None)
    call("sup_perman", C.c_void_p(P), 0, 6, 99, 0, None, C.byref(out), None)
    call("sup_perman", C.c_void_p(P), 0, 6, 0, 99, None, C.byref(out), None)
    call("sup_perman", C.c_void_p(P), 0, 6, 0, 0, None, None, None)
    call("sup_partial", C.c_void_p(P), 0, 6, 0, C.c_uint64(5), C.c_uint64(3), None, C.byref(out), None)
    call("sup_perman_shard", C.c_void_p(P), 0, 6, 0, 3, 2, None, C.byref(out), None)
    call("sup_perman_shard", C.c_void_p(P), 0, 6, 0, -1, 2, None, C.byref(out), None)
    # exact path: too-small output buffer, non-integer entries
    buf = C.create_string_buffer(4)
    call("sup_perman_exact", C.c_void_p(P), 0, 6, None, 1, buf, C.c_size_t(2), None)
    half = np.full((6, 6), 0.5)
    buf = C.create_string_buffer(600)
    call("sup_perman_exact", C.c_void_p(half.ctypes.data), 0, 6, None, 1, buf, C.c_size_t(600), None)
    call("sup_perman_exact", None, 0, 6, None, 1, buf, C.c_size_t(600), None)
    # readers and preprocessing
    call("sup_read_matrix", b"/nonexistent/file", 0, C.byref(C.c_void_p()), C.byref(C.c_int()),
         C.byref(C.c_int()), C.byref(C.c_int()))
    call("sup_read_mtx", b"/nonexistent/file.mtx", 0, C.byref(C.c_void_p()), C.byref(C.c_int()),
         C.byref(C.c_int()), C.byref(C.c_int()))
    call("sup_sort_order", None, 0, 6, None)
    call("sup_skip_order", C.c_void_p(P), 0, 0, None, None)
    call("sup_nw_start", None, 0, 6, None, None)
    call("sup_count_nnz", C.c_void_p(P), 0, 65, C.byref(C.c_int()))
    print("ok", len(codes))
""")


def test_malformed_calls_return_codes_not_crashes(sup):
    r = subprocess.run([sys.executable, "-c", f"ROOT = {ROOT!r}\n" + CHILD], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "")))
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.strip().startswith("ok")
