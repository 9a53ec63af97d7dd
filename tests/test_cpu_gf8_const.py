"""The compile-time GF(2^8) field of the bit-sliced tile (leopard_amd/csrc/
gf8_const.h, every multiplier of k_ff8_bs_slab is an XOR network compiled from
it) against the host library's tables (gf_tables.cpp), the oracle's, and the
reference's own LogLUT / ExpLUT / FFTSkew read out of oracle/_ref (the reference
compiled from its sources; LeopardFF8.cpp:136-194, 496-531).  CPU only: the
header is compiled here by g++ into a small dump program."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle_lib as ol

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def const_tables(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("gf8") / "gf8_const_dump")
    subprocess.run([gxx, "-std=c++17", "-O1", "-I", os.path.join(REPO, "leopard_amd", "csrc"),
                    os.path.join(HERE, "gf8_const", "gf8_const_dump.cpp"), "-o", exe], check=True)
    lines = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")
    log, exp, skew = (np.array([int(v) for v in lines[i].split()], dtype=np.int64) for i in range(3))
    mats = [int(v) for v in lines[3].split()]
    assert len(log) == 256 and len(exp) == 256 and len(skew) == 255 and len(mats) == 256
    return log, exp, skew, mats


def _mul(log, exp, a, c):
    """a * c with the oracle's tables (LeopardFF8.cpp:141-154 MultiplyLog)."""
    if a == 0 or c == 0:
        return 0
    s = int(log[a]) + int(log[c])
    return int(exp[(s + (s >> 8)) & 255])


def test_logs_and_exps_match_host_library_and_oracle(const_tables):
    log, exp, _, _ = const_tables
    assert np.array_equal(log, ol.oracle_table(False, 0).astype(np.int64))
    assert np.array_equal(exp, ol.oracle_table(False, 1).astype(np.int64))
    import leopard_amd
    assert np.array_equal(log, leopard_amd.table(8, 0).astype(np.int64))
    assert np.array_equal(exp, leopard_amd.table(8, 1).astype(np.int64))


def test_skews_are_the_reference_fft_skews(const_tables):
    """gf8_const keeps skews as elements; the reference (and gf_tables.cpp)
    keep their logs, 255 standing for the zero element."""
    log, exp, skew, _ = const_tables
    ref_logs = ol.oracle_table(False, 2).astype(np.int64)
    as_elements = np.where(ref_logs == 255, 0, exp[np.minimum(ref_logs, 255)])
    assert np.array_equal(skew, as_elements)
    import leopard_amd
    assert np.array_equal(ref_logs, leopard_amd.table(8, 2).astype(np.int64))


def test_multiply_matrices_are_the_field_multiply(const_tables):
    """Bit 8 i + j of gf8_matrix(c) is bit i of (1 << j) * c; by linearity the
    matrix applied to the bits of any x gives x * c (checked for all x, c)."""
    log, exp, _, mats = const_tables
    for c in range(256):
        m = mats[c]
        cols = [sum(((m >> (8 * i + j)) & 1) << i for i in range(8)) for j in range(8)]
        for j in range(8):
            assert cols[j] == _mul(log, exp, 1 << j, c), (c, j)
        for x in range(256):
            y = 0
            for j in range(8):
                if (x >> j) & 1:
                    y ^= cols[j]
            assert y == _mul(log, exp, x, c), (x, c)


def _ref_static_table(name, count, dtype):
    """A static table of the compiled reference, located through the symbol
    table (the library's own leo_init_ anchors the load address)."""
    so = ol.REF_SO
    nm = shutil.which("nm")
    if nm is None or not os.path.exists(so):
        pytest.skip("compiled reference (oracle/_ref) or nm not available")
    syms = {}
    for line in subprocess.run([nm, so], check=True, capture_output=True, text=True).stdout.splitlines():
        p = line.split()
        if len(p) == 3:
            syms[p[2]] = int(p[0], 16)
    ref = ol.reference()
    assert ref is not None
    base = ctypes.cast(ref.lib.leo_init_, ctypes.c_void_p).value - syms["leo_init_"]
    addr = base + syms[name]
    return np.ctypeslib.as_array((dtype * count).from_address(addr)).copy()


def test_tables_match_the_compiled_reference(const_tables):
    log, exp, skew, _ = const_tables
    ref = ol.reference()
    if ref is None:
        pytest.skip("compiled reference (oracle/_ref) not built")
    # the reference builds its tables in leo_init (CpuCodec called it)
    ref_log = _ref_static_table("_ZN7leopard3ff8L6LogLUTE", 256, ctypes.c_uint8).astype(np.int64)
    ref_exp = _ref_static_table("_ZN7leopard3ff8L6ExpLUTE", 256, ctypes.c_uint8).astype(np.int64)
    ref_skew = _ref_static_table("_ZN7leopard3ff8L7FFTSkewE", 255, ctypes.c_uint8).astype(np.int64)
    assert np.array_equal(log, ref_log)
    assert np.array_equal(exp, ref_exp)  # incl. the wrap ExpLUT[kModulus] = ExpLUT[0] (LeopardFF8.cpp:191)
    assert np.array_equal(skew, np.where(ref_skew == 255, 0, exp[np.minimum(ref_skew, 255)]))
