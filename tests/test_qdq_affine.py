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


def _join_ref(y, r, s3, z3, sr, zr, so):
    """The streaming kernel's fused join (out zero point 0) in its fp32 op
    order: sat(rne(((y - z3) s3 + (r - zr) sr) * fp32(1/so)))."""
    inv = F32(1) / F32(so)
    sm = ((y - F32(z3)) * F32(s3) + (r - F32(zr)) * F32(sr)).astype(F32)
    return np.clip(np.rint((sm * inv).astype(F32)), 0, 255)


def test_join_affine_is_exact_on_every_byte_pair(lib):
    """qcn_join_affine (the ResNet join's one form in conv1x1_stream_kernel):
    whenever a form is returned, rne(fma(y, a, fma(r, b, c))) equals the
    kernel's join on all 65536 (y3, identity) pairs; found for most layers."""
    y = np.arange(256, dtype=F32)[:, None]
    r = np.arange(256, dtype=F32)[None, :]
    rng = np.random.default_rng(11)
    found = 0
    n = 40
    for _ in range(n):
        s3 = F32(10 ** rng.uniform(-2.5, -1))
        sr = F32(s3 * 2 ** rng.uniform(-1.5, 1.5))
        so = F32(max(s3, sr) * 2 ** rng.uniform(0, 1.5))
        z3, zr = int(rng.integers(40, 220)), int(rng.integers(0, 8))
        out = (C.c_float * 3)()
        rc = lib.qcn_join_affine(C.c_float(s3), z3, C.c_float(sr), zr, C.c_float(so), out)
        assert rc in (0, 1)
        if rc == 0:
            continue
        found += 1
        a, b, c = (np.float64(out[i]) for i in range(3))
        inner = (r.astype(np.float64) * b + c).astype(F32)   # fma(r, b, c), one rounding
        v = (y.astype(np.float64) * a + inner.astype(np.float64)).astype(F32)
        got = np.clip(np.rint(v), 0, 255)
        want = _join_ref(y, r, s3, z3, sr, zr, so)
        assert np.array_equal(got, want), (s3, z3, sr, zr, so)
    assert found >= 0.75 * n, found
