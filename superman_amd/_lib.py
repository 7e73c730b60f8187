"""ctypes binding of the C ABI in include/superman.h (libsuperman_hip.so).

The shared library is built in-tree by ``superman_amd/csrc/Makefile`` (hipcc,
gfx950).  ``load()`` builds it on first use when it is missing, and raises
(never silently degrades) when it cannot be built or loaded.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "lib", "libsuperman_hip.so")
PERMAN_BIN = os.path.join(PKG_DIR, "bin", "perman")

SUP_OK = 0
ERRORS = {
    -1: "SUP_EINVAL",
    -2: "SUP_ENODEV",
    -3: "SUP_EHIP",
    -4: "SUP_ERCCL",
    -5: "SUP_ENOMEM",
    -6: "SUP_EIO",
    -7: "SUP_EUNSUPPORTED",
}
SUP_INT32, SUP_FLOAT32, SUP_FLOAT64 = 0, 1, 2
KERNEL_DENSE, KERNEL_SPARYSER, KERNEL_SKIPPER, KERNEL_DENSE_PLAIN, KERNEL_SEGMENTED, KERNEL_DENSE_LDS = 0, 1, 2, 3, 4, 5
SCHED_SINGLE, SCHED_STATIC, SCHED_CHUNKS, SCHED_MANUAL = 0, 1, 2, 3

# Every symbol include/superman.h declares (checked by tests/test_capi.py).
EXPORTS = [
    "sup_opts_init", "sup_abi_version", "sup_last_error", "sup_device_count", "sup_rccl_devices", "sup_device_checks", "sup_device_warmup", "sup_kernel_time",
    "sup_perman", "sup_partial", "sup_perman_cpu", "sup_nw_start", "sup_perman_shard", "sup_plan_info",
    "sup_prepare", "sup_plan_key", "sup_perman_exact", "sup_perman_reduced_exact", "sup_perman_quad",
    "sup_perman_reduced_quad",
    "sup_gpu_perman64_xshared_coalescing_mshared",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpu",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpu_manual_distribution",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse_manual_distribution",
    "sup_gpu_perman64_xshared_coalescing_mshared_sparse",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpu_sparse",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_sparse",
    "sup_gpu_perman64_xshared_coalescing_mshared_skipper",
    "sup_gpu_perman64_xshared_coalescing_mshared_multigpucpu_chunks_skipper",
    "sup_read_matrix", "sup_free", "sup_count_nnz", "sup_compress",
    "sup_sort_order", "sup_skip_order", "sup_read_mtx",
    "sup_reduce_opts_init", "sup_decompose", "sup_perman_reduced", "sup_approx", "sup_grid_graph",
]


class SupOpts(C.Structure):
    _fields_ = [
        ("gpu_num", C.c_int), ("device_id", C.c_int), ("threads", C.c_int),
        ("cpu_worker", C.c_int), ("grid_dim", C.c_int), ("block_dim", C.c_int),
        ("walk_log2", C.c_int), ("chunk_log2", C.c_int), ("use_rccl", C.c_int),
        ("verbose", C.c_int), ("jit", C.c_int), ("checkpoint", C.c_char_p), ("timing", C.c_int),
    ]


class SupReduceOpts(C.Structure):
    _fields_ = [
        ("compress", C.c_int), ("scale_threshold", C.c_double), ("min_n", C.c_int),
        ("max_deg", C.c_int), ("preprocessing", C.c_int),
    ]


class SupApproxResult(C.Structure):
    _fields_ = [
        ("mean", C.c_double), ("std_error", C.c_double), ("zero_fraction", C.c_double),
        ("samples", C.c_uint64), ("kernel_ms", C.c_double), ("wall_ms", C.c_double),
        ("devices", C.c_int), ("reserved_", C.c_int), ("cpu_blocks", C.c_int64),
    ]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved_"}


# int (*sup_leaf_fn)(const double* a, int n, void* user, double* out_perm)
LEAF_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int, C.c_void_p, C.POINTER(C.c_double))


class SupStats(C.Structure):
    _fields_ = [
        ("kernel_ms", C.c_double), ("wall_ms", C.c_double),
        ("gray_steps", C.c_uint64), ("visited_steps", C.c_uint64),
        ("devices_used", C.c_int), ("lane_bits", C.c_int), ("walk_bits", C.c_int),
        ("grid", C.c_int), ("chunks_done_cpu", C.c_int), ("partials", C.c_double * 16),
        ("walk_kind", C.c_int), ("leaves", C.c_int), ("est_ops_per_step", C.c_double),
        ("jit_ms", C.c_double), ("items_resumed", C.c_int), ("seg_cached_bits", C.c_int16),
        ("seg_pair_bits", C.c_int16),
    ]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_ if f != "partials"}
        d["partials"] = list(self.partials[: max(1, self.devices_used)])
        return d


class SupError(RuntimeError):
    def __init__(self, code: int, what: str, msg: str):
        super().__init__(f"{what}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None


def build(quiet: bool = True) -> None:
    """Compile the gfx950 engine in-tree (make -C superman_amd/csrc)."""
    jobs = str(min(16, os.cpu_count() or 4))
    r = subprocess.run(["make", "-C", CSRC, "-j", jobs], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("building libsuperman_hip.so failed:\n" + r.stdout[-4000:] + r.stderr[-4000:])
    if not quiet:
        print(r.stdout)


def load() -> C.CDLL:
    """Load libsuperman_hip.so (building it first if absent)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH) or not os.path.exists(PERMAN_BIN):
            build()
        lib = C.CDLL(LIB_PATH)
        _declare(lib)
        if lib.sup_abi_version() != 10:
            raise RuntimeError("libsuperman_hip.so ABI version mismatch")
        _lib = lib
        return lib


def _declare(lib: C.CDLL) -> None:
    P, I, D = C.c_void_p, C.c_int, C.c_double
    lib.sup_opts_init.argtypes = [C.POINTER(SupOpts)]
    lib.sup_opts_init.restype = None
    lib.sup_abi_version.restype = I
    lib.sup_last_error.restype = C.c_char_p
    lib.sup_device_count.argtypes = [C.POINTER(I)]
    lib.sup_rccl_devices.argtypes = [I, C.POINTER(I)]
    lib.sup_device_checks.restype = C.c_uint64
    lib.sup_device_warmup.argtypes = [I, I, I]
    lib.sup_kernel_time.restype = I
    lib.sup_kernel_time.argtypes = [I, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    lib.sup_perman.argtypes = [P, I, I, I, I, C.POINTER(SupOpts), C.POINTER(D), C.POINTER(SupStats)]
    lib.sup_partial.argtypes = [P, I, I, I, C.c_uint64, C.c_uint64, C.POINTER(SupOpts), C.POINTER(D),
                                C.POINTER(SupStats)]
    lib.sup_perman_cpu.argtypes = [P, I, I, I, I, C.POINTER(D), C.POINTER(SupStats)]
    lib.sup_perman_exact.argtypes = [P, I, I, C.POINTER(SupOpts), I, C.c_char_p, C.c_size_t, C.POINTER(SupStats)]
    lib.sup_perman_quad.argtypes = [P, I, I, C.POINTER(SupOpts), I, C.POINTER(D), C.POINTER(D), C.POINTER(SupStats)]
    lib.sup_perman_shard.argtypes = [P, I, I, I, I, I, C.POINTER(SupOpts), C.POINTER(D), C.POINTER(SupStats)]
    lib.sup_plan_info.argtypes = [P, I, I, I, C.POINTER(SupOpts), C.POINTER(I), P, C.POINTER(I), C.POINTER(I),
                                  C.POINTER(I), C.POINTER(I), C.POINTER(D)]
    lib.sup_prepare.argtypes = [P, I, I, I, C.POINTER(SupOpts), C.POINTER(I), C.POINTER(C.c_double)]
    lib.sup_plan_key.argtypes = [P, I, I, I, C.POINTER(SupOpts), C.POINTER(C.c_uint64)]
    lib.sup_nw_start.argtypes = [P, I, I, C.POINTER(D), C.POINTER(D)]
    lib.sup_read_matrix.argtypes = [C.c_char_p, I, C.POINTER(P), C.POINTER(I), C.POINTER(I), C.POINTER(I)]
    lib.sup_free.argtypes = [P]
    lib.sup_free.restype = None
    lib.sup_count_nnz.argtypes = [P, I, I, C.POINTER(I)]
    lib.sup_compress.argtypes = [P, I, I, P, P, P, P, P, P]
    lib.sup_sort_order.argtypes = [P, I, I, P]
    lib.sup_skip_order.argtypes = [P, I, I, P, P]
    lib.sup_approx.argtypes = [P, I, I, I, C.c_uint64, I, I, C.c_uint64, C.POINTER(SupOpts), I,
                               C.POINTER(SupApproxResult)]
    lib.sup_grid_graph.argtypes = [I, I, C.POINTER(C.POINTER(C.c_int)), C.POINTER(I)]
    lib.sup_read_mtx.argtypes = [C.c_char_p, I, C.POINTER(P), C.POINTER(I), C.POINTER(I), C.POINTER(I)]
    lib.sup_reduce_opts_init.argtypes = [C.POINTER(SupReduceOpts)]
    lib.sup_reduce_opts_init.restype = None
    lib.sup_decompose.argtypes = [P, I, I, C.POINTER(SupReduceOpts), LEAF_FN, P, C.POINTER(D), C.POINTER(I)]
    lib.sup_perman_reduced_exact.argtypes = [P, I, I, C.POINTER(SupOpts), I, C.POINTER(SupReduceOpts), C.c_char_p,
                                             C.c_size_t, C.POINTER(SupStats)]
    lib.sup_perman_reduced_quad.argtypes = [P, I, I, C.POINTER(SupOpts), I, C.POINTER(SupReduceOpts), C.POINTER(D),
                                            C.POINTER(D), C.POINTER(SupStats)]
    lib.sup_perman_reduced.argtypes = [P, I, I, I, I, C.POINTER(SupOpts), I, C.POINTER(SupReduceOpts),
                                       C.POINTER(D), C.POINTER(SupStats)]
    for name in EXPORTS:
        if name not in ("sup_opts_init", "sup_free", "sup_last_error", "sup_reduce_opts_init"):
            getattr(lib, name).restype = I


def check(rc: int, what: str) -> None:
    if rc != SUP_OK:
        msg = _lib.sup_last_error().decode(errors="replace") if _lib is not None else ""
        raise SupError(rc, what, msg)
