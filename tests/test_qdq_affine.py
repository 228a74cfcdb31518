"""CPU: the one-fma form of the QDQ hand-off (qcn_qdq_affine, the constants
the conv epilogues use when ConvEpi::qdq == 2) against the oracle's
dequantize -> ReLU -> quantize_per_tensor (oracle/qref.py A7 / A1; reference
custom_quantization_model.py:41-45, :237-252).

For every integer r = rint(ab) the requant can produce, the layer's u8 output
is q1 = clamp(r + y_zp, lo, 255) and the next stub's input is
g(q1) = quantize_per_tensor(relu(dequantize(q1, s1, z1)), s2, z2); the form
must give rne_sat_u8(med3(fma(r, qa, qb), glo, ghi)) == g(q1) for all of them
(r far outside [lo - y_zp, 255 - y_zp] included: the clamps must hold there).
Host-only: no device work is called."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import qref
from tests import netfix

F32 = np.float32


@pytest.fixture(scope="module")
def lib():
    from qconvnet import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libqconvnet.so missing — run __graft_entry__.build()")
    return _lib.load()


def _form(lib, s1, z1, s2, z2, y_zp, lo):
    from qconvnet import ops
    q = ops.qdq_struct(s1, z1, s2, z2)
    out = (C.c_float * 4)()
    rc = lib.qcn_qdq_affine(C.byref(q), int(y_zp), int(lo), out)
    assert rc in (0, 1)
    return (F32(out[0]), F32(out[1]), F32(out[2]), F32(out[3])) if rc == 1 else None


def _fma32(r, a, b):
    # exact fused multiply-add rounded once to fp32: r (|r| < 2^10) * a (24-bit
    # mantissa) is exact in fp64, and so is the sum with b for these magnitudes
    return (r.astype(np.float64) * np.float64(a) + np.float64(b)).astype(F32)


def _check(form, s1, z1, s2, z2, y_zp, lo):
    qa, qb, glo, ghi = form
    r = np.arange(-600, 601, dtype=np.int64)
    q1 = np.clip(r + y_zp, lo, 255)
    want = qref.quantize_per_tensor(np.maximum(qref.dequantize(q1, s1, z1), F32(0)), s2, z2)
    v = np.minimum(np.maximum(_fma32(r, qa, qb), glo), ghi)
    got = np.clip(np.rint(v), 0, 255).astype(np.uint8)   # v_cvt_pk_u8_f32: RNE, saturate
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (f"r={r[bad[:5]]} got={got[bad[:5]]} want={want[bad[:5]]}", form)


def test_qdq_affine_on_the_config2_fixture_layers(lib):
    """Every hand-off of the pinned config-2 net (conv1..conv6 -> next stub)
    has an exact one-fma form, and it is exact."""
    spec = netfix.qdq_spec(netfix.load())
    found = 0
    for i in range(1, 7):
        e = spec[f"conv{i}"]
        s2, z2 = e["next"]
        form = _form(lib, e["s_y"], e["z_y"], s2, z2, e["z_y"], 0)
        if form is not None:
            found += 1
            _check(form, e["s_y"], e["z_y"], s2, z2, e["z_y"], 0)
    assert found == 6


def test_qdq_affine_random_qparams(lib):
    """Random scales / zero points (ratios s1/s2 from 1/64 to 64, every
    floor): whenever a form is returned it is exact, and one is found for
    nearly all of them."""
    rng = np.random.default_rng(7)
    found = 0
    n = 400
    for _ in range(n):
        s1 = F32(10.0 ** rng.uniform(-4, 0))
        s2 = F32(s1 * 2.0 ** rng.uniform(-6, 6))
        z1, z2, y_zp = (int(v) for v in rng.integers(0, 256, 3))
        lo = y_zp if rng.random() < 0.3 else 0
        form = _form(lib, s1, z1, s2, z2, y_zp, lo)
        if form is not None:
            found += 1
            _check(form, s1, z1, s2, z2, y_zp, lo)
    assert found >= 0.95 * n, found


def test_qdq_affine_exact_ties(lib):
    """Scale ratios that put (q1 - z1) s1 / s2 exactly on .5 (round half to
    even before z2 is added): the form must reproduce the tie-breaking or
    decline."""
    for s1, s2 in ((0.5, 1.0), (0.25, 0.5), (1.5, 1.0), (0.125, 0.25), (3.0, 2.0)):
        for z1 in (0, 3, 128):
            for z2 in (0, 1, 7, 128):
                form = _form(lib, F32(s1), z1, F32(s2), z2, z1, 0)
                if form is not None:
                    _check(form, F32(s1), z1, F32(s2), z2, z1, 0)
