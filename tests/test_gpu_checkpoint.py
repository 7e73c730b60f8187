"""Checkpoint / resume of the chunk queue (the dynamic scheduler's
chunk ids allow it; the reference has none).  sup_opts.checkpoint (CLI
--checkpoint, Python perman(checkpoint=...)) records every finished queue item
of a -p6 / -p8 call; a later call with the file takes the recorded items
instead of walking them.  The item partials are exact fp64 bit patterns folded
by the same pairwise tree, so a resumed run returns the uninterrupted bits."""
import os
import struct
import subprocess

import pytest

import bench
from conftest import ROOT, fixture_path

pytestmark = pytest.mark.gpu


def _read(path):
    lines = open(path).read().splitlines()
    head = lines[0].split()
    assert head[:2] == ["supckpt", "2"]  # plan key, library build id, toolchain, c0, c1, item, nitems
    nitems = int(head[8])
    parts, vis = [None] * nitems, [0] * nitems
    for ln in lines[1:]:
        i, bits, v = ln.split()
        parts[int(i)] = struct.unpack("<d", int(bits, 16).to_bytes(8, "little"))[0]
        vis[int(i)] = int(v)
    return lines, parts, vis


def test_checkpoint_records_and_resumes(sup, tmp_path):
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    full = sup.perman(a, 6)
    ck = str(tmp_path / "run.ckpt")
    r1, st1 = sup.perman(a, 6, checkpoint=ck, return_stats=True)
    assert r1 == full and st1["items_resumed"] == 0
    lines, parts, vis = _read(ck)
    nitems = len(parts)
    assert nitems >= 8 and None not in parts and sum(vis) == 1 << 29
    assert -2.0 * bench.pairwise(parts) == full  # the recorded partials are the sum, item by item (n even)

    # interrupted: the first k items recorded, then a torn line
    k = nitems // 2
    with open(ck, "w") as f:
        f.write("\n".join(lines[: 1 + k]) + "\n" + lines[1 + k][:9])
    r2, st2 = sup.perman(a, 6, checkpoint=ck, return_stats=True)
    assert r2 == full and st2["items_resumed"] == k
    assert st2["visited_steps"] == 1 << 29
    _, parts2, _ = _read(ck)
    assert parts2 == parts  # complete again, same bits

    # recorded items are taken, not walked again: a doctored partial shows in the result
    j = 3
    with open(ck, "w") as f:
        f.write(lines[0] + "\n" + f"{j} {struct.unpack('<Q', struct.pack('<d', 0.0))[0]:016x} 0\n")
    r3, st3 = sup.perman(a, 6, checkpoint=ck, return_stats=True)
    doctored = list(parts)
    doctored[j] = 0.0
    assert st3["items_resumed"] == 1 and r3 == -2.0 * bench.pairwise(doctored) and r3 != full

    # another computation's file is refused; so is a schedule without the chunk queue
    with pytest.raises(sup.SupError, match="another computation"):
        sup.perman(0.5 * a, 6, checkpoint=ck)
    with pytest.raises(sup.SupError, match="chunk queue"):
        sup.perman(a, 4, checkpoint=str(tmp_path / "other.ckpt"))
    # an empty file (created beforehand) starts afresh
    open(ck, "w").close()
    r4, st4 = sup.perman(a, 6, checkpoint=ck, return_stats=True)
    assert r4 == full and st4["items_resumed"] == 0 and _read(ck)[1] == parts


def test_checkpoint_sparse_skipper_and_hybrid(sup, tmp_path):
    a, _, _ = sup.read_matrix(fixture_path("int__30_0.20_0"))
    k = sup.skip_order(a)[0]
    want = sup.perman(k, 8, sparse=True, jit=-1)
    ck = str(tmp_path / "skip.ckpt")
    # the item size is part of the header: fix it (2^9 wave-chunks, 16 items at n = 30) to resume on
    # another device count (the default size follows the device count)
    assert sup.perman(k, 8, sparse=True, jit=-1, checkpoint=ck, chunk_log2=9) == want
    lines, parts, _ = _read(ck)
    with open(ck, "w") as f:
        f.write("\n".join(lines[:3]) + "\n")
    # resumed by the devices and the hybrid CPU worker together (two logical devices on GPU 0)
    os.environ["SUP_DEVICE_MAP"] = "0,0"
    try:
        got, st = sup.perman(k, 8, sparse=True, jit=-1, checkpoint=ck, chunk_log2=9, gpu_num=2, cpu=True,
                             threads=4, return_stats=True)
        with pytest.raises(sup.SupError, match="another computation"):  # default item size for 2 devices
            sup.perman(k, 8, sparse=True, jit=-1, checkpoint=ck, gpu_num=2)
    finally:
        del os.environ["SUP_DEVICE_MAP"]
    assert got == want and st["items_resumed"] == 2


def test_checkpoint_cli(sup, tmp_path):
    exe = os.path.join(ROOT, "superman_amd", "bin", "perman")
    f = fixture_path("double__30_0.50_0")
    ck = str(tmp_path / "cli.ckpt")

    def run(*extra):
        out = subprocess.run([exe, "-f", f, "-g", "-p6", "-d1", *extra], capture_output=True, text=True,
                             timeout=300, check=True).stdout
        return [ln for ln in out.splitlines() if ln.startswith("Permanent:")][0]

    plain = run()
    assert run("--checkpoint", ck) == plain
    assert run("--checkpoint", ck, "-v") == plain  # every item resumed from the file
    assert open(ck).read().startswith("supckpt 2 ")


def test_checkpoint_from_another_build_refused(sup, tmp_path):
    """The header names the library build (ELF build id) and the hiprtc
    toolchain beside the plan: a file written by another binary is refused
    rather than mixed into a run that claims the uninterrupted bits."""
    a, _, _ = sup.read_matrix(fixture_path("double__30_0.50_0"))
    ck = str(tmp_path / "run.ckpt")
    sup.perman(a, 6, checkpoint=ck)
    lines = open(ck).read().splitlines()
    head = lines[0].split()
    assert int(head[3], 16) != 0  # the library carries a build id
    head[3] = "%016x" % (int(head[3], 16) ^ 1)
    open(ck, "w").write("\n".join([" ".join(head)] + lines[1:]) + "\n")
    with pytest.raises(sup.SupError):
        sup.perman(a, 6, checkpoint=ck)
