"""CPU tier: the C-ABI shared library loads, exports every symbol the headers
declare, and keeps the reference's validation order and result codes
(leopard.cpp:123-344) for everything decided before touching a GPU."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    names = set()
    for h in ("leopard.h", "leopard_amd.h"):
        with open(os.path.join(REPO, "include", h)) as f:
            text = f.read()
        for m in re.finditer(r"LEO_EXPORT[^;]*?\b(leo_\w+)\s*\(", text, re.S):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_the_reference_abi():
    names = set(_declared_symbols())
    for n in ("leo_init_", "leo_result_string", "leo_encode_work_count", "leo_encode", "leo_decode_work_count",
              "leo_decode"):
        assert n in names


@pytest.mark.parametrize("name", _declared_symbols())
def test_library_exports_symbol(name):
    import leopard_amd
    lib = ctypes.CDLL(leopard_amd.LIB_PATH)
    assert hasattr(lib, name)


def test_work_counts_match_reference_formulas():
    import leopard_amd as leo
    import oracle_lib as ol
    o = ol.oracle()
    for k in (1, 2, 3, 100, 128, 129, 1000, 32768, 65535):
        for r in (1, 2, 3, 64, 100, 128, 200, 32768):
            if r > k:
                continue
            assert leo.leo_encode_work_count(k, r) == o.encode_work_count(k, r)
            assert leo.leo_decode_work_count(k, r) == o.decode_work_count(k, r)


def test_result_strings():
    import leopard_amd as leo
    assert leo.leo_result_string(0) == "Operation succeeded"
    assert leo.leo_result_string(-7) == "Call leo_init() first"
    assert leo.leo_result_string(-3) == "Buffer size must be a multiple of 64 bytes"
    assert leo.leo_result_string(5) == "Unknown"


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_gpu(), reason="CPU-only behaviour")
def test_no_gpu_fails_loudly():
    import leopard_amd as leo
    assert leo.leo_init(3) == leo.LeopardResult.InvalidInput  # version mismatch first
    assert leo.leo_init() == leo.LeopardResult.Platform
    buf = (ctypes.c_uint8 * 64)()
    p = ctypes.addressof(buf)
    # size/count/null checks precede the init check (leopard.cpp:131-141)
    assert leo.leo_encode(65, 2, 2, 4, [p, p], [p] * 4) == leo.LeopardResult.InvalidSize
    assert leo.leo_encode(64, 2, 3, 4, [p, p], [p] * 4) == leo.LeopardResult.InvalidCounts
    assert leo.leo_encode(64, 2, 2, 4, None, [p] * 4) == leo.LeopardResult.InvalidInput
    assert leo.leo_encode(64, 2, 2, 4, [p, p], [p] * 4) == leo.LeopardResult.CallInitialize
    assert leo.leo_decode(64, 2, 2, 4, [p, None], [p, p], [p] * 4) == leo.LeopardResult.CallInitialize
    assert leo.leo_decode(64, 2, 2, 4, [p, None], None, [p] * 4) == leo.LeopardResult.InvalidInput
