"""ctypes binding of libqconvnet.so (the C ABI declared in include/qconvnet.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
convnet-quantization_amd/csrc``).  There is no fallback: if the shared object
is missing, importing the compute path raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QCN_LIB", os.path.join(_HERE, "libqconvnet.so"))

QCN_OK = 0
QCN_ERR_ARG = -1
QCN_ERR_UNSUPPORTED = -2
QCN_ERR_HIP = -3
_ERRS = {QCN_ERR_ARG: "invalid argument", QCN_ERR_UNSUPPORTED: "unsupported shape",
         QCN_ERR_HIP: "HIP runtime error"}


class QcnError(RuntimeError):
    pass


class QDQ(C.Structure):
    """qcn_qdq_t"""
    _fields_ = [("s1", C.c_float), ("z1", C.c_int32), ("inv2", C.c_float), ("z2", C.c_int32)]


class ConvLayer(C.Structure):
    """qcn_conv_layer_t"""
    _fields_ = [("w", C.c_void_p), ("u", C.c_void_p), ("v", C.c_void_p), ("mult", C.c_void_p),
                ("corr", C.c_void_p), ("x_zp", C.c_int32), ("y_zp", C.c_int32), ("relu", C.c_int32),
                ("qdq", C.POINTER(QDQ))]


vp = C.c_void_p
i32 = C.c_int
i64 = C.c_longlong
f32 = C.c_float

# name -> (restype, argtypes)
SIGNATURES = {
    "qcn_version": (i32, []),
    "qcn_quantize_f32_u8": (i32, [vp, vp, i32, i32, i32, i32, i32, f32, i32, vp]),
    "qcn_dequantize_u8_f32": (i32, [vp, vp, i64, f32, i32, vp]),
    "qcn_minmax_reset": (i32, [vp, vp]),
    "qcn_minmax_f32": (i32, [vp, i64, vp, vp]),
    "qcn_maxpool2x2_u8_nhwc": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "qcn_argmax_f32": (i32, [vp, i32, i32, vp, vp]),
    "qcn_channel_affine_f32": (i32, [vp, i32, i32, vp, vp, i32, vp, vp]),
    "qcn_conv3x3_packed_size": (i32, [i32, i32]),
    "qcn_pack_conv3x3_weight": (i32, [vp, i32, i32, vp, vp]),
    "qcn_pack_conv1_weight": (i32, [vp, i32, vp, vp]),
    "qcn_conv3x3_u8s8_nhwc": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, i32,
                                    i32, C.POINTER(QDQ), vp, vp]),
    "qcn_convnet_convs_f32_nchw": (i32, [vp, i32, f32, i32, C.POINTER(ConvLayer), vp, vp, vp, i32, vp]),
    "qcn_convnet_convs_form": (i32, [i32, f32, i32, C.POINTER(ConvLayer), i32]),
    "qcn_convs36_u8s8": (i32, [vp, i32, C.POINTER(ConvLayer), vp, vp, i32, vp]),
    "qcn_conv1_f32_nchw": (i32, [vp, i32, i32, f32, i32, vp, vp, vp, vp, vp, i32, i32,
                                 C.POINTER(QDQ), vp, vp, vp]),
    "qcn_conv12_fused_f32_nchw": (i32, [vp, i32, f32, i32, vp, vp, vp, vp, vp, i32, i32,
                                        C.POINTER(QDQ), i32, vp, vp, vp, vp, vp, i32, i32,
                                        C.POINTER(QDQ), vp, vp]),
    "qcn_linear_u8s8": (i32, [vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, i32, vp, vp, f32, vp]),
    "qcn_classifier_workspace_size": (i64, [i32, i32]),
    "qcn_pack_fc_kmajor": (i32, [vp, i32, i32, vp]),
    "qcn_qdq_affine": (i32, [C.POINTER(QDQ), i32, i32, vp]),
    "qcn_join_affine": (i32, [f32, i32, f32, i32, f32, vp]),
    "qcn_conv3x3_pair_u8s8": (i32, [vp, i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, i32,
                                    C.POINTER(QDQ), vp, i32, vp, vp, vp, vp, i32, i32,
                                    C.POINTER(QDQ), i32, vp, vp]),
    "qcn_conv3x3_u8s8_kmajor": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, i32,
                                      i32, vp, vp]),
    "qcn_classifier_u8s8": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, vp, i32, i32, vp, i32, vp, vp,
                                  vp, i32, i32, f32, vp, vp, vp, vp, vp]),
    "qcn_dq_bn_q_u8": (i32, [vp, i64, i32, f32, i32, vp, vp, i32, f32, i32, vp, vp]),
    "qcn_dq_bn_relu_maxpool_f32": (i32, [vp, i32, i32, i32, i32, f32, i32, vp, vp, vp, f32, i32, vp,
                                         vp]),
    "qcn_qdq_join_f32": (i32, [vp, f32, i32, vp, vp, vp, f32, i32, vp, vp, vp, i64, i32, vp, f32, i32,
                               vp, vp]),
    "qcn_avgpool_f32_nhwc": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "qcn_classifier_qdq_u8s8": (i32, [vp, i32, i32, vp, i32, vp, vp, vp, vp, i32, f32, vp, i32, vp,
                                      vp, vp, vp, vp]),
    "qcn_pack_conv_weight_kmajor": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "qcn_resnet_stem_fused": (i32, [vp, i32, i32, i32, f32, i32, vp, i32, vp, vp, vp, vp, i32, i32,
                                    vp, vp]),
    "qcn_conv_u8s8_nhwc": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32, i32,
                                 vp, vp, vp, vp, i32, i32, vp, vp]),
    "qcn_conv_gemm_u8s8_nhwc": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, i32, i32, i32, i32, i32,
                                      i32, vp, vp, vp, vp, i32, i32, vp, f32, f32, i32, f32, i32,
                                      vp, vp]),
    "qcn_conv1x1_join_reduce_u8s8_nhwc": (i32, [vp, i32, i32, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, vp,
                                                f32, f32, i32, f32, i32, vp, vp, i32, vp, vp, vp, vp, i32,
                                                i32, vp, vp]),
    "qcn_add_relu_u8": (i32, [vp, f32, i32, vp, f32, i32, i64, f32, i32, i32, vp, vp]),
    "qcn_maxpool3x3s2_u8_nhwc": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "qcn_stem_pack_f32_nchw": (i32, [vp, i32, i32, i32, f32, i32, vp, vp]),
    "qcn_avgpool_u8_nhwc": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "qcn_linear_dynamic_workspace_size": (i64, [i32, i32]),
    "qcn_linear_dynamic_f32": (i32, [vp, i32, i32, vp, i32, vp, i32, vp, vp, i32, vp, vp, vp]),
    "qcn_linear_dynamic_range_f32": (i32, [vp, i32, i32, vp, i32, vp, i32, vp, vp, i32, vp, vp, vp,
                                           vp]),
    "qcn_linear_f32": (i32, [vp, i32, i32, vp, i32, vp, i32, vp, vp]),
}

_lib = None


def load():
    """Load the shared library once and declare every entry point."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise QcnError(f"libqconvnet.so not found at {LIB_PATH}; run __graft_entry__.build() "
                       "(there is no CPU fallback for the int8 path)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != QCN_OK:
        raise QcnError(f"{what}: {_ERRS.get(rc, 'error')} ({rc})")
    return rc
