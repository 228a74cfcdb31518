/*
 * qconvnet.h — C ABI of the MI355X (gfx950) int8 ConvNet inference path.
 *
 * One shared library, libqconvnet.so, built from
 * the HIP sources in convnet-quantization_amd/csrc/.  Every compute entry point:
 *   - takes caller-owned DEVICE pointers (e.g. torch tensors' data_ptr()),
 *     explicit shapes and quantization parameters, and an explicit HIP
 *     stream (hipStream_t passed as void*; NULL = default stream);
 *   - allocates nothing and never synchronizes (safe inside hipGraph capture);
 *   - returns 0 (QCN_OK) or a negative status; no exceptions cross the ABI.
 * The qcn_pack_* functions work on HOST memory (one-time weight packing).
 *
 * The reference (his0si/ConvNet-Quantization) has no FFI: its hot path is the
 * torch.ao / FBGEMM arithmetic behind its duck-typed model objects.  Each entry
 * below names the reference interface it replaces (file:line in
 * /root/reference unless prefixed torch/, which is the torch 2.10 wheel).
 * Numerics are bit-exact with torch.ao's fbgemm engine on the integer path
 * (see oracle/qref.py and tests/golden/).
 */
#ifndef QCONVNET_H
#define QCONVNET_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QCN_OK 0
#define QCN_ERR_ARG (-1)          /* invalid argument / shape                     */
#define QCN_ERR_UNSUPPORTED (-2)  /* shape combination has no kernel              */
#define QCN_ERR_HIP (-3)          /* HIP launch / runtime error                   */

/* Per-layer QDQ hand-off (CustomQuantizedConv2d chain): after requantizing to
 * (scale s1, zero point z1), dequantize, ReLU, and quantize with the next
 * layer's input qparams (inv2 = fp32(1/scale2), z2).  Replaces the fp32
 * DeQuantStub -> F.relu -> [pool] -> QuantStub sequence of
 * models/custom_quantization_model.py:41-45, :237-252. */
typedef struct qcn_qdq_t {
  float s1;
  int32_t z1;
  float inv2;
  int32_t z2;
} qcn_qdq_t;

/* One conv of SimpleConvNet for qcn_convnet_convs_f32_nchw: packed weights
 * (qcn_pack_conv1_weight for conv1, qcn_pack_conv3x3_weight otherwise), the
 * requant constants, the input / output zero points, ReLU and the optional
 * QDQ hand-off into the next layer. */
typedef struct qcn_conv_layer_t {
  const int8_t* w;
  const float* u;
  const float* v;
  const float* mult;
  const int32_t* corr;
  int32_t x_zp;
  int32_t y_zp;
  int32_t relu;
  const qcn_qdq_t* qdq;
} qcn_conv_layer_t;

/* Library version (major*10000 + minor*100 + patch). */
int qcn_version(void);

/* A1 — aten::quantize_per_tensor (QuantStub once converted,
 * models/custom_quantization_model.py:42,55,234):
 *   q = clamp(zp + rne(x * fp32(1/scale)), 0, 255).
 * x is fp32 [n,c,h,w] NCHW; q is u8, NHWC when nhwc_out != 0 else NCHW. */
int qcn_quantize_f32_u8(const float* x, uint8_t* q, int n, int c, int h, int w, int nhwc_out,
                        float scale, int zero_point, void* stream);

/* A7 — aten::dequantize (DeQuantStub, custom_quantization_model.py:44,57,260):
 *   x = fp32(scale) * fp32(q - zp). */
int qcn_dequantize_u8_f32(const uint8_t* q, float* x, long long count, float scale,
                          int zero_point, void* stream);

/* A2 — MinMaxObserver.forward (torch/ao/quantization/observer.py:558-569):
 * running [min, max] of fp32 data, reduced on the device.  minmax points to 2
 * device floats; qcn_minmax_reset writes [+inf, -inf]. */
int qcn_minmax_reset(float* minmax, void* stream);
int qcn_minmax_f32(const float* x, long long count, float* minmax, void* stream);

/* A10 — nn.MaxPool2d(2, 2) on u8 NHWC (baseline_model.py:17,25,33). */
int qcn_maxpool2x2_u8_nhwc(const uint8_t* x, int n, int h, int w, int c, uint8_t* y,
                           void* stream);

/* A11 — argmax over the last axis, ties -> lowest index (torch.argmax /
 * topk(1), utils/model_evaluator.py:36,96,160). */
int qcn_argmax_f32(const float* x, int rows, int cols, long long* idx, void* stream);

/* Inference BatchNorm1d (+ReLU) on fp32 [rows, cols] (bn7 of the reference's
 * StaticPTQModel between its dynamic fc1 and fc2, models/static_ptq_model.py:
 * 19-34 over baseline_model.py:80-82): y = fma(x, alpha[c], beta[c]), then
 * max(y, 0) when relu, in ATen's CPU op order (alpha / beta from the host,
 * qconvnet.quant.bn_eval_affine).  cols % 4 == 0, 16-B aligned pointers. */
int qcn_channel_affine_f32(const float* x, int rows, int cols, const float* alpha,
                           const float* beta, int relu, float* y, void* stream);

/* A5/A6 weight packing (host).  w_oihw is torch's s8 [cout][cin][3][3].
 * out receives qcn_conv3x3_packed_size(cin, cout) bytes; wsum[cout] receives
 * sum_k w (for the activation zero-point correction). */
int qcn_conv3x3_packed_size(int cin, int cout);
int qcn_pack_conv3x3_weight(const int8_t* w_oihw, int cout, int cin, int8_t* out, int32_t* wsum);
int qcn_pack_conv1_weight(const int8_t* w_oihw, int cout, int8_t* out, int32_t* wsum);

/* A5/A6/A10 — QuantizedConv2d / QuantizedConvReLU2d (fbgemm), 3x3, pad 1,
 * stride 1, optionally followed by a fused 2x2 max-pool and a per-layer QDQ
 * hand-off (qdq may be NULL).  Replaces the conv of CustomQuantizedConv2d
 * (custom_quantization_model.py:43) and the FX/eager full-int8 conv.
 *   x: u8 NHWC [nimg,h,w,cin] (zero point x_zp);  y: u8 NHWC.
 *   u, v, mult: fp32 [cout] epilogue constants (t = fmaf(u,v,acc); ab = t*mult)
 *   corr: int32 [cout] = (128 - x_zp) * wsum  (activations enter the MFMA as
 *   q - 128). */
int qcn_conv3x3_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                          const int8_t* w_packed, int cout, const float* u, const float* v,
                          const float* mult, const int32_t* corr, int y_zp, int relu, int pool,
                          const qcn_qdq_t* qdq, uint8_t* y, void* stream);

/* A1 + conv1 .. conv6 of SimpleConvNet (baseline_model.py:60-72; per-layer
 * QDQ form custom_quantization_model.py:233-255) in ONE persistent launch:
 * fp32 NCHW [nimg,3,32,32] in (quantized with in_scale / in_zp ==
 * layers[0].x_zp), conv6's pooled output into a6: chunk-major
 * ([128][nimg][32], the classifier head's input) when kmajor != 0, NHWC
 * [nimg,4,4,256] otherwise; a2 ([nimg,16,16,64]) and a4 ([nimg,8,8,128]) are
 * written on the way.  Each workgroup carries its own
 * images through all six convs, so the results are those of
 * qcn_conv12_fused_f32_nchw + two qcn_conv3x3_pair_u8s8 launches bit for
 * bit.  By batch, with C = the device's CUs:
 *   nimg <= C        one image per workgroup (convnet_convs_sm_kernel);
 *   C < nimg < 4 C   QCN_ERR_UNSUPPORTED (the caller launches the three kernels);
 *   nimg >= 4 C      one persistent workgroup per CU, when conv3..conv6 are all
 *                    on the FBGEMM fast epilogue or all on the one-fma QDQ form
 *                    (else QCN_ERR_UNSUPPORTED).
 * layers[i].x_zp must be conv i-1's output zero point (its QDQ hand-off's z2
 * when it has one): QCN_ERR_ARG otherwise. */
int qcn_convnet_convs_f32_nchw(const float* x, int nimg, float in_scale, int in_zp,
                               const qcn_conv_layer_t* layers, uint8_t* a2, uint8_t* a4, uint8_t* a6,
                               int kmajor, void* stream);

/* A5+A6+A10 x4 — conv3 .. conv6 of SimpleConvNet (baseline_model.py:20-33,
 * :64-75) in one persistent launch of 256-thread workgroups (one wave per
 * SIMD, 64-cout x 256-pixel wave tiles, r06): a2 u8 NHWC [nimg,16,16,64] in
 * (qcn_conv12_fused_f32_nchw's output), a4 ([nimg,8,8,128]) written on the
 * way, conv6's pooled output into a6 as qcn_convnet_convs_f32_nchw writes it
 * (chunk-major when kmajor).  layers: the four layers conv3 .. conv6
 * (layers[0].x_zp = conv2's output zero point).  Bit-exact with the pair
 * launches.  QCN_ERR_UNSUPPORTED unless conv3..conv6 are all on the FBGEMM
 * fast epilogue or all on the one-fma QDQ form. */
int qcn_convs36_u8s8(const uint8_t* a2, int nimg, const qcn_conv_layer_t* layers, uint8_t* a4, uint8_t* a6,
                     int kmajor, void* stream);

/* Host query (no launch): which form qcn_convnet_convs_f32_nchw takes for
 * these arguments on the current device — 1 one image per workgroup, 2 the
 * persistent form, or the error it would return (QCN_ERR_UNSUPPORTED,
 * QCN_ERR_ARG, QCN_ERR_HIP). */
int qcn_convnet_convs_form(int nimg, float in_scale, int in_zp, const qcn_conv_layer_t* layers, int kmajor);

/* A1+A5+A6 fused — QuantStub + conv1(+ReLU) of SimpleConvNet
 * (baseline_model.py:13, :60): fp32 NCHW [nimg,3,hw,hw] in, quantized with
 * (in_scale, in_zp), 3x3 conv to 64 channels, u8 NHWC out.  q_in (optional,
 * may be NULL) receives the quantized input, u8 NHWC. */
int qcn_conv1_f32_nchw(const float* x, int nimg, int hw, float in_scale, int in_zp,
                       const int8_t* w1_packed, const float* u, const float* v, const float* mult,
                       const int32_t* corr, int y_zp, int relu, const qcn_qdq_t* qdq, uint8_t* y,
                       uint8_t* q_in, void* stream);

/* A1+A5+A6+A10 fused — QuantStub + conv1(+ReLU) + conv2(+ReLU) + 2x2 max-pool
 * of SimpleConvNet's first block (baseline_model.py:13-18, :60-63): fp32 NCHW
 * [nimg,3,32,32] in, u8 NHWC [nimg,16,16,64] out; conv1's activation stays in
 * LDS.  Parameters as qcn_conv1_f32_nchw (conv1: z1 = its output zero point,
 * qdq1 its optional hand-off) and qcn_conv3x3_u8s8_nhwc (conv2: x2_zp = its
 * input zero point). */
int qcn_conv12_fused_f32_nchw(const float* x, int nimg, float in_scale, int in_zp,
                              const int8_t* w1_packed, const float* u1, const float* v1,
                              const float* mult1, const int32_t* corr1, int z1, int relu1,
                              const qcn_qdq_t* qdq1, int x2_zp, const int8_t* w2_packed,
                              const float* u2, const float* v2, const float* mult2,
                              const int32_t* corr2, int y_zp, int relu2, const qcn_qdq_t* qdq2,
                              uint8_t* y, void* stream);

/* Two convolutions of one SimpleConvNet block in one launch: conv A
 * (cin -> cmid, no pool) then conv B (cmid -> cout, fused 2x2 max-pool).  A's
 * output never leaves LDS; the results are those of two qcn_conv3x3_u8s8_nhwc
 * calls (A's u8 output zero point zmid is B's input zero point, or qdqa->z2 in
 * QDQ mode; qdqa / qdqb may be NULL).  y: u8 NHWC [nimg, hw/2, hw/2, cout], or chunk-major like
 * qcn_conv3x3_u8s8_kmajor when kmajor != 0.  Supported: (hw 16, 64 -> 128 ->
 * 128) and (hw 8, 128 -> 256 -> 256) — SimpleConvNet conv3+conv4 and
 * conv5+conv6; QCN_ERR_UNSUPPORTED otherwise. */
int qcn_conv3x3_pair_u8s8(const uint8_t* x, int nimg, int hw, int cin, int x_zp,
                          const int8_t* wa_packed, int cmid, const float* ua, const float* va,
                          const float* multa, const int32_t* corra, int zmid, int relua,
                          const qcn_qdq_t* qdqa, const int8_t* wb_packed, int cout, const float* ub,
                          const float* vb, const float* multb, const int32_t* corrb, int y_zp,
                          int relub, const qcn_qdq_t* qdqb, int kmajor, uint8_t* y, void* stream);

/* A5/A6 as above, but y is written chunk-major for the classifier head:
 * y[f / 32][nimg][32] with f the NHWC flatten index of one image's output
 * (oh * ow * cout bytes).  Supported: the 8x8 layers with cout == 256
 * (SimpleConvNet conv5/conv6), QCN_ERR_UNSUPPORTED otherwise. */
int qcn_conv3x3_u8s8_kmajor(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                            const int8_t* w_packed, int cout, const float* u, const float* v,
                            const float* mult, const int32_t* corr, int y_zp, int relu, int pool,
                            uint8_t* y, void* stream);

/* A9 — quantized Linear / LinearReLU (fbgemm), static qparams:
 * fc1/fc2 of SimpleConvNet (baseline_model.py:38,40).
 *   x: u8 [m,k] (zero point x_zp); w: s8 [n,k] row-major; y: u8 [m,n].
 *   y_deq (optional) receives fp32 (y - y_zp) * y_scale  (DeQuantStub). */
int qcn_linear_u8s8(const uint8_t* x, int m, int k, int x_zp, const int8_t* w, int n,
                    const float* u, const float* v, const float* mult, const int32_t* corr,
                    int y_zp, int relu, uint8_t* y, float* y_deq, float y_scale, void* stream);

/* A9 x 2 + A7 — the static classifier head in two launches: fc1 (+ReLU)
 * u8 x s8 -> u8 [m, n1] as a 4-way split-K GEMM into an int32 workspace, then
 * one wave per row finishes fc1 (requant) and computes fc2 (n2 <= 16) and its
 * DeQuantStub.  Same results as qcn_linear_u8s8(fc1) followed by
 * qcn_linear_u8s8(fc2, y_deq) — fc2's input zero point is y1_zp, fc2's
 * correction is applied exactly in the finisher (no corr2 argument).
 * x and w1 are CHUNK-MAJOR: x[k/32][m][32] (qcn_conv3x3_u8s8_kmajor writes
 * conv6's output that way), w1[k/32][n1][32] (qcn_pack_fc_kmajor).
 * corr1 = (128 - x_zp) * sum_k w1[f][k].  Supported: m % 128 == 0, n1 == 512,
 * k % 1024 == 0, n2 <= 16 (QCN_ERR_UNSUPPORTED otherwise).  workspace: device
 * memory of qcn_classifier_workspace_size(m, n1) bytes (the int32 split-K
 * partials; no initialisation needed); one workspace per stream the head runs
 * on concurrently. */
long long qcn_classifier_workspace_size(int m, int n1);
/* Host: s8 [n][k] row-major -> [k/32][n][32] (k % 32 == 0). */
int qcn_pack_fc_kmajor(const int8_t* w, int n, int k, int8_t* out);
/* Host: the QDQ hand-off (qcn_qdq_t) after a requant to (y_zp, lo) in its
 * one-fma form.  With r = rint(ab) of the requant, the layer output is
 * q1 = clamp(r + y_zp, lo, 255) and the next stub's input g(q1); on success
 * (returns 1) out[4] = {qa, qb, glo, ghi} with
 *   g(clamp(r + y_zp, lo, 255)) == rne_sat_u8(med3(fma(r, qa, qb), glo, ghi))
 * for every integer r (checked in fp32 over all r with q1 in [lo, 255]);
 * returns 0 when no exact form was found (the conv epilogues then run the
 * general requant + qdq sequence).  The conv launchers apply it themselves;
 * exported for the host tests (no device work). */
int qcn_qdq_affine(const qcn_qdq_t* q, int y_zp, int lo, float* out);
/* Host: the fused residual join of the ResNet bottleneck (out zero point 0,
 * custom_quantization_model.py:94-101) in its one form: on success (returns
 * 1) out[3] = {a, b, c} with
 *   sat(rne(((y - y_zp) y_scale + (r - r_zp) r_scale) * fp32(1/out_scale)))
 *     == sat(rne(fma(y, a, fma(r, b, c))))
 * for all 256 x 256 byte pairs (y, r) in the kernel's fp32 op order; 0 when
 * no exact form was found (the streaming kernel then keeps the sequence).
 * Applied by qcn_conv_gemm_u8s8_nhwc itself; exported for the host tests. */
int qcn_join_affine(float y_scale, int y_zp, float r_scale, int r_zp, float out_scale, float* out);
int qcn_classifier_u8s8(const uint8_t* x, int m, int k, const int8_t* w1, int n1, const float* u1,
                        const float* v1, const float* mult1, const int32_t* corr1, int y1_zp,
                        int relu1, const int8_t* w2, int n2, const float* u2, const float* v2,
                        const float* mult2, int y2_zp, int relu2, float y2_scale, void* workspace,
                        uint8_t* y1, uint8_t* y2, float* y2_deq, void* stream);

/* QDQ classifier head (CustomQuantizedSimpleConvNet, BASELINE config 2;
 * custom_quantization_model.py:218-219, 256-258): fc1's QuantStub -> int8
 * Linear -> requant to (y1_scale, y1_zp) (no ReLU in the int8 op) ->
 * DeQuantStub -> F.relu (fp32) -> fc2 as an fp32 nn.Linear (w2 fp32 [n2][n1],
 * b2 fp32 [n2] or NULL) -> y2 fp32 [m][n2].  y1 (optional) receives fc1's u8
 * output.  Same split-K first launch, layouts, envelope and workspace as
 * qcn_classifier_u8s8; fc2's fp32 sums run in a different order from a CPU
 * sgemm (the QDQ tests bound the difference). */
int qcn_classifier_qdq_u8s8(const uint8_t* x, int m, int k, const int8_t* w1, int n1,
                            const float* u1, const float* v1, const float* mult1,
                            const int32_t* corr1, int y1_zp, float y1_scale, const float* w2,
                            int n2, const float* b2, void* workspace, uint8_t* y1, float* y2,
                            void* stream);

/* A8 — quantized::linear_dynamic (DynamicQuantizedLinear of
 * models/static_ptq_model.py:28-32 and models/dynamic_ptq_model.py:302-306):
 * per-call activation qparams from the batch min/max (ChooseQuantizationParams,
 * qrange [0,127] when reduce_range), quantize, u8 x s8 GEMM,
 * y = fmaf(fp32(acc), fp32(s_x * s_w), bias).  w_scale holds 1 (per-tensor) or
 * n (per-channel) floats; bias may be NULL.  workspace: >= 64 bytes of device
 * memory + m*k bytes (quantized activations). */
long long qcn_linear_dynamic_workspace_size(int m, int k);
int qcn_linear_dynamic_f32(const float* x, int m, int k, const int8_t* w, int n,
                           const float* w_scale, int per_channel, const int32_t* wsum,
                           const float* bias, int reduce_range, float* y, void* workspace,
                           void* stream);

/* A8 with the activation range supplied by the caller: minmax points to 2
 * device floats [min, max] — e.g. the all-reduced range of every rank's shard,
 * which makes a sharded dynamic Linear batch-exact.  Otherwise
 * identical to qcn_linear_dynamic_f32. */
int qcn_linear_dynamic_range_f32(const float* x, int m, int k, const int8_t* w, int n,
                                 const float* w_scale, int per_channel, const int32_t* wsum,
                                 const float* bias, int reduce_range, const float* minmax,
                                 float* y, void* workspace, void* stream);

/* fp32 Linear (fc2 of CustomQuantizedSimpleConvNet stays fp32,
 * custom_quantization_model.py:219): y = x @ w^T + b, with optional ReLU on x
 * (relu_in) applied on load. */
int qcn_linear_f32(const float* x, int m, int k, const float* w, int n, const float* b,
                   int relu_in, float* y, void* stream);

/* ---- ResNet-style bottleneck blocks (config 5) ----------
 * CustomQuantizedBottleneck / CustomQuantizedResNet50
 * (models/custom_quantization_model.py:60-148): 1x1, 3x3 (strided) and 1x1
 * downsample convs, the fp32-domain residual add + ReLU (:94-101), the stem
 * conv + maxpool, the global average pool and the fc classifier. */

/* Host: s8 OIHW [cout][cin][kh][kw] -> chunk-major [kh*kw*cin/32][cout][32]
 * (K ordered (r, s, c)); wsum[cout] = sum of each filter.  cin % 32 == 0. */
int qcn_pack_conv_weight_kmajor(const int8_t* w_oihw, int cout, int cin, int kh, int kw,
                                int8_t* out, int32_t* wsum);
/* Quantized Conv2d(+ReLU) (QuantizedConv2d / QuantizedConvReLU2d with
 * per-channel or per-tensor weights) on u8 NHWC, any kernel / stride /
 * padding; requant as qcn_conv3x3_u8s8_nhwc (A6).  cin % 32 == 0,
 * cout % 64 == 0; corr = (128 - x_zp) * wsum.  Output [n][oh][ow][cout]. */
int qcn_conv_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                       const int8_t* w_packed, int cout, int kh, int kw, int stride_h,
                       int stride_w, int pad_h, int pad_w, const float* u, const float* v,
                       const float* mult, const int32_t* corr, int y_zp, int relu, uint8_t* y,
                       void* stream);
/* Same conv as qcn_conv_u8s8_nhwc on the LDS-tiled implicit-GEMM kernel
 * (256-pixel x 128/64-channel tiles, LDS-DMA im2col).  With resid != NULL the
 * residual join is fused into the epilogue (the conv must have relu == 0):
 * y3 = requant(acc) with (y_scale, y_zp), then
 * y = quantize(relu(y_scale*(y3-y_zp) + r_scale*(resid-r_zp)), out_scale, out_zp)
 * — bit-identical to qcn_conv_u8s8_nhwc followed by qcn_add_relu_u8. */
int qcn_conv_gemm_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                            const int8_t* w_packed, int cout, int kh, int kw, int stride_h,
                            int stride_w, int pad_h, int pad_w, const float* u, const float* v,
                            const float* mult, const int32_t* corr, int y_zp, int relu,
                            const uint8_t* resid, float y_scale, float r_scale, int r_zp,
                            float out_scale, int out_zp, uint8_t* y, void* stream);
/* The bottleneck's expand + residual join (qcn_conv_gemm_u8s8_nhwc with
 * resid, 1x1, cin 64 -> cout 256) with the NEXT block's reduce conv (1x1,
 * stride 1, 256 -> cout2 in {64, 128}, input zero point out_zp) fused: y is
 * the joined block output (u8 NHWC [n][h][w][256], the next identity), y2 the
 * reduce's output [n][h][w][cout2] (FBGEMM requant with u2/v2/mult2/corr2,
 * y2_zp, relu2).  Bit-identical to the two separate launches; replaces
 * custom_quantization_model.py:89-101 of block i followed by :81-83 (conv1,
 * bn1, relu) of block i + 1.  QCN_ERR_UNSUPPORTED for other shapes. */
int qcn_conv1x1_join_reduce_u8s8_nhwc(const uint8_t* x, int nimg, int h, int w, int cin, int x_zp,
                                      const int8_t* w_packed, int cout, const float* u, const float* v,
                                      const float* mult, const int32_t* corr, int y_zp, const uint8_t* resid,
                                      float y_scale, float r_scale, int r_zp, float out_scale, int out_zp,
                                      uint8_t* y, const int8_t* w2_packed, int cout2, const float* u2,
                                      const float* v2, const float* mult2, const int32_t* corr2, int y2_zp,
                                      int relu2, uint8_t* y2, void* stream);
/* Residual join (custom_quantization_model.py:94-101 then the next stage's
 * QuantStub): y = quantize(relu?(fp32(sa*(a-za)) + fp32(sb*(b-zb))), s_out, z_out). */
int qcn_add_relu_u8(const uint8_t* a, float sa, int za, const uint8_t* b, float sb, int zb,
                    long long count, float s_out, int z_out, int relu, uint8_t* y, void* stream);
/* nn.MaxPool2d(3, 2, padding=1) on u8 NHWC (c % 16 == 0). */
int qcn_maxpool3x3s2_u8_nhwc(const uint8_t* x, int nimg, int h, int w, int c, uint8_t* y,
                             void* stream);
/* QuantStub on fp32 NCHW [n][3][h][w] fused with the row im2col of the 7x7 /
 * stride-2 / pad-3 stem: y[n][h][ow][32], byte 3*s+ch = q(x[n][ch][iy][2*ox-3+s]),
 * zero point outside the image and in bytes 21..31.  ow = (w-1)/2 + 1. */
int qcn_stem_pack_f32_nchw(const float* x, int nimg, int h, int w, float scale, int zp, uint8_t* y,
                           void* stream);
/* The whole ResNet stem in one launch: QuantStub (scale, zp) on fp32 NCHW
 * [n][3][h][w] -> 7x7/2 pad-3 conv 3->64 (w_packed = stem_weight_rows packed
 * k-major, [7][64][32]; u/v/mult/corr and y_zp/relu as qcn_conv_gemm_u8s8_nhwc)
 * -> MaxPool2d(3, 2, padding=1) -> u8 NHWC [n][h/4][w/4][64].  Bit-identical
 * to qcn_stem_pack_f32_nchw + qcn_conv_gemm_u8s8_nhwc (7x1, strides (2,1), pad
 * (3,0)) + qcn_maxpool3x3s2_u8_nhwc; replaces the reference's
 * conv1/bn1/relu/maxpool of custom_quantization_model.py:117-141 after its
 * QuantStub.  h == w in {224, 64}, cout == 64, else QCN_ERR_UNSUPPORTED. */
int qcn_resnet_stem_fused(const float* x, int nimg, int h, int w, float scale, int zp,
                          const int8_t* w_packed, int cout, const float* u, const float* v,
                          const float* mult, const int32_t* corr, int y_zp, int relu, uint8_t* y,
                          void* stream);
/* AdaptiveAvgPool2d(1) on u8 NHWC [nimg][hw][c] -> [nimg][c], quantization
 * parameters kept (torch's quantized adaptive_avg_pool2d, the avgpool of a
 * static-int8 ResNet ahead of its fc): y = clamp(x_zp + rne(fp32(sum_q -
 * hw*x_zp) * fp32(1/hw)), 0, 255).  c % 4 == 0. */
int qcn_avgpool_u8_nhwc(const uint8_t* x, int nimg, int hw, int c, int x_zp, uint8_t* y,
                        void* stream);

/* ---- SURVEY §8(f)2 in the reference's own semantics ----------------------
 * CustomQuantizedBottleneck / CustomQuantizedResNet50 with live per-layer
 * stubs (models/custom_quantization_model.py:34-45, 60-143): fp32 BN / ReLU /
 * max-pool / residual add / avg-pool between int8 convs
 * (qcn_conv_gemm_u8s8_nhwc, requant to each conv's own output qparams, no
 * ReLU).  All maps NHWC, C % 4 == 0; alpha / beta are BN's eval constants
 * (ATen: alpha = fp32(fp32(1/sqrt(var+eps)) * gamma), beta = fmaf(-mean,
 * alpha, bias); the map is fmaf(x, alpha, beta)); every quantize is
 * zp + rint(x * fp32(1/s)) clamped to [0, 255]; ReLU keeps -0.0 (torch.relu).
 * Pointers: u8 4-B aligned, fp32 maps and alpha / beta 16-B aligned. */
/* conv -> DeQuantStub -> BN -> [ReLU] -> next conv's QuantStub (u8 -> u8). */
int qcn_dq_bn_q_u8(const uint8_t* y, long long count, int c, float s, int z, const float* alpha,
                   const float* beta, int relu, float s_next, int z_next, uint8_t* out,
                   void* stream);
/* Stem: conv -> DeQuantStub -> BN -> ReLU -> MaxPool2d(3, 2, 1): fp32
 * [n][(h-1)/2+1][(w-1)/2+1][c] (the first block's input and identity), plus,
 * when out_q is not NULL, that map quantized for block 0's QuantStubs. */
int qcn_dq_bn_relu_maxpool_f32(const uint8_t* y, int n, int h, int w, int c, float s, int z,
                               const float* alpha, const float* beta, float* out, float s_next,
                               int z_next, uint8_t* out_q, void* stream);
/* Residual join (:92-101): out = relu(bn3(dq(y3)) + identity), identity =
 * bn_d(dq(yd)) (downsample conv, yd != NULL) or the fp32 block input idf;
 * fp32 out, plus out_q (optional) quantized for the next block's stubs. */
int qcn_qdq_join_f32(const uint8_t* y3, float s3, int z3, const float* a3, const float* b3,
                     const uint8_t* yd, float sd, int zd, const float* ad, const float* bd,
                     const float* idf, long long count, int c, float* out, float s_next, int z_next,
                     uint8_t* out_q, void* stream);
/* AdaptiveAvgPool2d(1) on fp32 NHWC: sequential fp32 sum over the window in
 * row-major order, then / (h*w) (ATen's channels-last kernel) -> [n][c]. */
int qcn_avgpool_f32_nhwc(const float* x, int n, int h, int w, int c, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QCONVNET_H */
