"""The C-ABI boundary: library loads, exports every symbol include/superman.h
declares, reports errors through codes + sup_last_error, and the GPU entry
points refuse to run without a device (no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, fixture_path


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "superman.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sup_[a-z0-9_]+)\s*\(", txt)))


def test_exports_every_declared_symbol(sup):
    lib = sup._lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(sup._lib.EXPORTS) == syms


def test_exports_visible_to_nm(sup):
    out = subprocess.run(["nm", "-D", "--defined-only", sup._lib.LIB_PATH], capture_output=True, text=True).stdout
    for s in header_symbols():
        assert re.search(rf"\bT {s}$", out, re.M), s


def test_library_holds_gfx950_code(sup):
    # the fat binary embeds code objects for amdgcn-amd-amdhsa--gfx950 only
    data = open(sup._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"--gfx906", b"--gfx90a", b"--gfx942"):
        assert other not in data


def test_error_codes(sup):
    lib = sup._lib.load()
    out = C.c_double()
    a = np.ones((3, 3))
    rc = lib.sup_perman_cpu(a.ctypes.data, 2, 0, 0, 1, C.byref(out), None)
    assert rc == -1 and b"outside" in lib.sup_last_error()
    rc = lib.sup_perman_cpu(a.ctypes.data, 2, 65, 0, 1, C.byref(out), None)
    assert rc == -1
    rc = lib.sup_perman_cpu(None, 2, 3, 0, 1, C.byref(out), None)
    assert rc == -1
    with pytest.raises(ValueError):
        sup.perman(np.ones((2, 3)))
    with pytest.raises(sup.SupError):
        sup.perman(np.ones((3, 3)), algo=9)


def test_walk_option_bounds(sup):
    # the kernels index the walk in 32 bits and pack walk-bit data for k < 32:
    # walk_log2 > 31 and chunk_log2 >= 63 are refused before any planning or
    # device work (so the check holds on a CPU-only host too)
    a = np.ones((44, 44))
    for kw in ({"walk_log2": 32}, {"walk_log2": 40}, {"walk_log2": -1}, {"chunk_log2": 63}, {"chunk_log2": -2}):
        with pytest.raises(sup.SupError) as e:
            sup.perman(a, **kw)
        assert e.value.code == -1 and ("walk_log2" in str(e.value) or "chunk_log2" in str(e.value)), kw
    with pytest.raises(sup.SupError) as e:
        sup.partial(a, 0, 1 << 20, walk_log2=32)
    assert e.value.code == -1
    # sup_perman_shard and sup_plan_key validate them too (n = 60 with
    # walk_log2 = 40 would give T = 1u << 40 in the kernels)
    b = np.ones((60, 60))
    for call in (lambda: sup.perman_shard(b, 0, 1, walk_log2=40), lambda: sup.plan_key(b, walk_log2=40),
                 lambda: sup.plan_info(b, walk_log2=40), lambda: sup.prepare(b, walk_log2=40)):
        with pytest.raises(sup.SupError) as e:
            call()
        assert e.value.code == -1 and "walk_log2" in str(e.value)


def test_fixed_walk_length_is_its_own_plan(sup, tmp_path):
    """A walk_log2 request equal to the default m is a fixed layout (the
    segmented planner keeps it) and must not share a plan-cache slot with the
    auto layout (which may lengthen m): after plan_info(mat), a fixed request
    gets the plan a fresh process gets."""
    a = sup.read_matrix(fixture_path("double__36_0.20_0"))[0]
    a = sup.sort_order(a)[0]
    L, m, h = sup.layout(36)
    auto = sup.plan_info(a, "seg")
    here = sup.plan_key(a, "seg", walk_log2=m)
    # the same compiler as this process (torch first resolves hiprtc to its own copy)
    code = ("import torch; " if "torch" in sys.modules else "") + (
            "import sys; sys.path.insert(0, {root!r}); import numpy as np, superman_amd as S; "
            "a = np.load({p!r}); print(S.plan_key(a, 'seg', walk_log2={m}))").format(root=ROOT, p=str(tmp_path / "a.npy"),
                                                                                      m=m)
    np.save(tmp_path / "a.npy", a)
    fresh = int(subprocess.run(["python3", "-c", code], capture_output=True, text=True, check=True,
                               env=dict(os.environ, SUP_JIT_CACHE_DIR="")).stdout.split()[-1])
    assert here == fresh
    info = sup.plan_info(a, "seg", walk_log2=m)
    assert info["m"] == m
    assert auto["m"] >= m  # the auto layout lengthens cheap walks (config 3: m 14)


def test_partial_range_validation(sup):
    if sup.device_count() > 0:
        pytest.skip("GPU present: covered by the gpu tests")
    with pytest.raises(sup.SupError) as e:
        sup.partial(np.ones((10, 10)), 3, 64)
    assert e.value.code == -1


def test_gpu_entry_points_fail_loudly_without_device(sup):
    if sup.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(sup.SupError) as e:
        sup.perman(np.ones((8, 8)), algo=4)
    assert e.value.code == -2  # SUP_ENODEV: never a silent CPU fallback
    with pytest.raises(sup.SupError):
        sup.gpu_perman64_xshared_coalescing_mshared_skipper(np.ones((8, 8)))


def test_cli_cpu_mode(sup):
    exe = sup._lib.PERMAN_BIN
    r = subprocess.run([exe, "-f", fixture_path("synth/12_0.50_int"), "-c", "-t", "4"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0].startswith("Result: parallel_perman64 ")
    val = float(lines[1].split()[1])
    a, _, _ = sup.read_matrix(fixture_path("synth/12_0.50_int"))
    assert val == sup.perman_cpu(a, "dense", 2)


def test_cli_errors_and_missing_file(sup):
    exe = sup._lib.PERMAN_BIN
    # -a without a GPU: the GPU estimators fail loudly (no CPU fallback); -c -a runs on the host
    r = subprocess.run([exe, "-f", fixture_path("synth/12_0.50_int"), "-a"], capture_output=True, text=True)
    if sup.device_count() == 0:
        assert r.returncode == 1 and "no HIP device" in r.stderr
    r = subprocess.run([exe, "-f", fixture_path("synth/12_0.50_int"), "-a", "-c", "-p1", "-x", "640"],
                       capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("Result: rasmussen ")
    r = subprocess.run([exe, "-c"], capture_output=True, text=True)
    assert r.returncode == 1 and "required" in r.stderr
    r = subprocess.run([exe, "-f", "/nonexistent", "-c"], capture_output=True, text=True)
    assert r.returncode == 1


def test_cli_sparse_cpu_ids(sup):
    exe = sup._lib.PERMAN_BIN
    f = fixture_path("synth/16_0.20_int")
    outs = {}
    for p, name in ((1, "parallel_perman64_sparse"), (2, "parallel_skip_perman64_w"),
                    (3, "parallel_skip_perman64_w_balanced")):
        r = subprocess.run([exe, "-f", f, "-c", "-s", "-r2", f"-p{p}", "-t2"], capture_output=True, text=True)
        assert r.returncode == 0 and r.stdout.startswith(f"Result: {name} "), r.stdout + r.stderr
        outs[p] = float(r.stdout.splitlines()[1].split()[1])
    assert abs(outs[1] - outs[3]) <= 1e-12 * abs(outs[1])


def test_rccl_devices_follow_a_permuted_map():
    """The -R combine's communicators, slot buffers and streams all sit on the
    physical device of each logical one (the slot buffers were
    allocated on the logical ids).  A permuted SUP_DEVICE_MAP maps through;
    a repeated physical id is refused; no map is the identity.  The map is read
    per call, so each case runs in a fresh process."""
    import subprocess
    import sys
    code = ("import superman_amd as S, sys\n"
            "try:\n    print(S.rccl_devices(int(sys.argv[1])))\n"
            "except S.SupError as e:\n    print('err', e.code)\n")
    cases = [("1,0", 2, "[1, 0]"), ("2,3,0,1", 4, "[2, 3, 0, 1]"), ("", 3, "[0, 1, 2]"), ("0,0", 2, "err -4")]
    for m, g, want in cases:
        env = dict(os.environ, SUP_DEVICE_MAP=m, PYTHONPATH=ROOT)
        r = subprocess.run([sys.executable, "-c", code, str(g)], capture_output=True, text=True, env=env,
                           timeout=60)
        assert r.stdout.strip() == want, (m, r.stdout, r.stderr)
