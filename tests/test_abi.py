"""CPU: the C-ABI library loads, exports every symbol include/qconvnet.h
declares, and its host-side (packing) entry points are correct.  No device
compute is called here."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "qconvnet.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(qcn_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from qconvnet import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libqconvnet.so missing — run __graft_entry__.build()")
    return _lib.load()


def test_every_declared_symbol_is_exported(lib):
    names = _declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert missing == []


def test_binding_covers_header():
    from qconvnet import _lib
    assert set(_declared()) == set(_lib.SIGNATURES)


def test_version(lib):
    assert lib.qcn_version() >= 100


def test_pack_conv3x3_layout(lib):
    from qconvnet import ops
    rng = np.random.default_rng(0)
    for cin, cout in ((64, 64), (128, 256), (3, 64), (48, 32)):
        w = rng.integers(-128, 128, (cout, cin, 3, 3)).astype(np.int8)
        packed, wsum = ops.pack_conv3x3(w)
        assert np.array_equal(wsum, w.reshape(cout, -1).astype(np.int64).sum(1))
        ohwi = w.transpose(0, 2, 3, 1).reshape(cout, 9, cin)
        if cin % 64 == 0 and cout % 64 == 0:
            # [chunk = tap*(cin/64) + cb][cout][64]
            p = packed.reshape(9, cin // 64, cout, 64)
            ref = ohwi.reshape(cout, 9, cin // 64, 64).transpose(1, 2, 0, 3)
            assert np.array_equal(p, ref)
        else:
            assert np.array_equal(packed.reshape(cout, 9, cin), ohwi)


def test_pack_conv1_layout(lib):
    from qconvnet import ops
    w = np.random.default_rng(1).integers(-128, 128, (64, 3, 3, 3)).astype(np.int8)
    packed, wsum = ops.pack_conv1(w)
    p = packed.reshape(64, 32)
    assert np.all(p[:, 27:] == 0)
    ref = w.transpose(0, 2, 3, 1).reshape(64, 27)  # k = tap*3 + c
    assert np.array_equal(p[:, :27], ref)
    assert np.array_equal(wsum, ref.astype(np.int64).sum(1))


def test_bad_arguments_return_status(lib):
    import ctypes as C
    assert lib.qcn_pack_conv3x3_weight(None, 64, 64, None, None) == -1
    assert lib.qcn_conv3x3_u8s8_nhwc(None, 1, 8, 8, 64, 0, None, 64, None, None, None, None, 0, 1,
                                     0, None, None, None) == -1
    assert lib.qcn_quantize_f32_u8(None, None, 1, 1, 1, 1, 0, C.c_float(1.0), 0, None) == -1
    assert lib.qcn_linear_u8s8(None, 1, 1, 0, None, 1, None, None, None, None, 0, 0, None, None,
                               C.c_float(1.0), None) == -1


def test_product_fails_loudly_without_library(monkeypatch, tmp_path):
    """The int8 path has no CPU fallback: a missing .so raises."""
    import importlib
    from qconvnet import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.QcnError):
        _lib.load()
    importlib.reload(_lib)
