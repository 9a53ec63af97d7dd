"""The drop-in boundary from a plain C program: tests/c_caller/leo_c_caller.c
includes include/leopard.h and is linked against libleopard_amd.so and
libleopard_amd.a (built by `make -C leopard_amd`), the way the reference's own
callers use the reference library (tests/benchmark.cpp:384-385, 421-428,
472-479; the reference ships a static lib, CMakeLists.txt:17-31)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as ol

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "c_caller", "bin")
CALLERS = ["leo_c_caller_so", "leo_c_caller_a"]


def _run(name, *args, timeout=120):
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        pytest.fail(f"{path} missing: build it with `make -C leopard_amd`")
    return subprocess.run([path, *map(str, args)], capture_output=True, text=True, timeout=timeout)


def _fields(out):
    res = {}
    for line in out.splitlines():
        key, _, val = line.partition(" ")
        res[key + (" " + val.split()[0] if key == "check" else "")] = val
    return res


def _gpu():
    from conftest import gpu_available
    return gpu_available()


@pytest.mark.parametrize("name", CALLERS)
def test_c_caller_links_and_validates(name):
    """Argument validation through the C ABI (leopard.cpp:131-140) and, with no
    gfx950 GPU, leo_init() = Leopard_Platform (-6) and a clean exit code 3."""
    p = _run(name, 10, 3, 64, 2)
    f = _fields(p.stdout)
    assert f["check invalid_size"].split()[-1] == "-3"
    assert f["check invalid_counts"].split()[-1] == "-4"
    assert f["check invalid_input"].split()[-1] == "-5"
    assert f["result_string"] == "Invalid counts provided"
    if not _gpu():
        assert f["init"] == "-6" and p.returncode == 3, p.stdout + p.stderr


def _pattern(k, b):
    i = np.arange(k, dtype=np.uint64)[:, None]
    j = np.arange(b, dtype=np.uint64)[None, :]
    return ((i * 131 + j * 7 + 3 + (j >> np.uint64(8)) * 29) & np.uint64(255)).astype(np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CALLERS)
@pytest.mark.parametrize("k,r,b,loss", [(100, 20, 1024, 20), (128, 128, 4096, 64), (1000, 200, 640, 200)])
def test_c_caller_roundtrip_on_gpu(name, k, r, b, loss):
    """The C program's host-buffer encode matches the oracle byte for byte
    (FNV-1a-64 of the recovery pieces) and its decode rebuilds the originals."""
    p = _run(name, k, r, b, loss)
    assert p.returncode == 0, p.stdout + p.stderr
    f = _fields(p.stdout)
    assert f["init"] == "0"
    expect = ol.oracle().encode(_pattern(k, b), r)
    h = 0xCBF29CE484222325
    for byte in expect.tobytes():
        h = ((h ^ byte) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    assert f["recovery_fnv"] == f"{h:016x}"
    assert "decode ok" in p.stdout
