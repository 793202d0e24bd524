// Anchor generation, training-target encoding and box decoding — the index/IoU work of
// efficientnet/utils/anchors.py.  Bit-exact with the reference's fp32 op sequence: no FMA
// contraction, correctly rounded division, argmax ties to the first index.
//
//   anchor boxes : Anchors._generate_boxes (anchors.py:47-84).  Centres follow tf.range's
//                  fp32 accumulation (start, start+delta, ...), box = centre -/+ fp32(half)
//   targets      : Anchors.generate_targets (anchors.py:91-138) with get_iou 'iou'
//                  (iou.py:27-69) and _boxes_encoder (anchors.py:219-243)
//   decode       : Anchors._boxes_decoder (anchors.py:245-274)
#pragma clang fp contract(off)
#include "common.hpp"

namespace edet {

__global__ void k_anchor_boxes(int fh, int fw, float sy, float dy, float sx, float dx, int A, const float* half,
                               float* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= fh * fw * A) return;
  const int a = i % A, hw = i / A, h = hw / fw, w = hw - h * fw;
  float yc = sy, xc = sx;
  for (int k = 0; k < h; ++k) yc = yc + dy;  // tf.range accumulates in the output dtype
  for (int k = 0; k < w; ++k) xc = xc + dx;
  const float hy = half[2 * a], hx = half[2 * a + 1];
  float* o = out + (size_t)i * 4;
  o[0] = yc - hy;
  o[1] = xc - hx;
  o[2] = yc + hy;
  o[3] = xc + hx;
}

__device__ __forceinline__ float iou_tf(const float* b1, const float* b2) {
  const float zero = 0.f;
  const float b1_w = fmaxf(zero, b1[3] - b1[1]), b1_h = fmaxf(zero, b1[2] - b1[0]);
  const float b2_w = fmaxf(zero, b2[3] - b2[1]), b2_h = fmaxf(zero, b2[2] - b2[0]);
  const float a1 = b1_w * b1_h, a2 = b2_w * b2_h;
  const float iy1 = fmaxf(b1[0], b2[0]), ix1 = fmaxf(b1[1], b2[1]);
  const float iy2 = fminf(b1[2], b2[2]), ix2 = fminf(b1[3], b2[3]);
  const float iw = fmaxf(zero, ix2 - ix1), ih = fmaxf(zero, iy2 - iy1);
  const float inter = iw * ih;
  const float uni = (a1 + a2) - inter;
  return (uni == 0.f) ? 0.f : inter / uni;  // divide_no_nan
}

__global__ void k_targets(const float* anchors, edet_pyramid p, int A, const float* gt, const int32_t* gt_cls,
                          const int32_t* n_gt, int max_gt, float thr, float* box_t, int32_t* cls_t, uint8_t* mask,
                          int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  int64_t rem = i;
  int seg = 0;
  int64_t abase = 0;
  for (; seg < p.nseg - 1; ++seg) {
    const int64_t cnt = (int64_t)p.batch * p.H[seg] * p.W[seg] * A;
    if (rem < cnt) break;
    rem -= cnt;
    abase += (int64_t)p.H[seg] * p.W[seg] * A;
  }
  const int hwa = p.H[seg] * p.W[seg] * A;
  const int n = (int)(rem / hwa);
  const int r = (int)(rem - (int64_t)n * hwa);  // hw * A + a
  const float* an = anchors + (abase + r) * 4;
  const int ng = n_gt[n];
  const float* g = gt + (size_t)n * max_gt * 4;
  int best = 0;
  float bv = 0.f;
  for (int k = 0; k < ng; ++k) {
    const float v = iou_tf(an, g + 4 * k);
    if (k == 0 || v > bv) { bv = v; best = k; }
  }
  const bool pos = ng > 0 && bv >= thr;
  const int64_t row = (int64_t)p.row_off[seg] * A + (int64_t)n * hwa + r;  // (pyramid row)*A + a
  float* bt = box_t + row * 4;
  if (pos) {
    const float* gb = g + 4 * best;
    const float ycenter_a = (an[2] + an[0]) / 2.0f, xcenter_a = (an[3] + an[1]) / 2.0f;
    float ha = an[2] - an[0], wa = an[3] - an[1];
    const float ycenter = (gb[2] + gb[0]) / 2.0f, xcenter = (gb[3] + gb[1]) / 2.0f;
    float h = gb[2] - gb[0], w = gb[3] - gb[1];
    const float eps = 1e-8f;
    ha = fmaxf(eps, ha); wa = fmaxf(eps, wa); h = fmaxf(eps, h); w = fmaxf(eps, w);
    bt[0] = (ycenter - ycenter_a) / ha;
    bt[1] = (xcenter - xcenter_a) / wa;
    bt[2] = logf(h / ha);
    bt[3] = logf(w / wa);
    cls_t[row] = gt_cls[(size_t)n * max_gt + best];
  } else {
    bt[0] = 0.f; bt[1] = 0.f; bt[2] = 0.f; bt[3] = 0.f;
    cls_t[row] = 0;
  }
  mask[row] = pos ? 1 : 0;
}

template <typename T>
__global__ void k_decode(const float* anchors, edet_pyramid p, int A, const T* rel, int ld, float* out,
                         int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  int64_t rem = i;
  int seg = 0;
  int64_t abase = 0;
  for (; seg < p.nseg - 1; ++seg) {
    const int64_t cnt = (int64_t)p.batch * p.H[seg] * p.W[seg] * A;
    if (rem < cnt) break;
    rem -= cnt;
    abase += (int64_t)p.H[seg] * p.W[seg] * A;
  }
  const int hwa = p.H[seg] * p.W[seg] * A;
  const int n = (int)(rem / hwa);
  const int r = (int)(rem - (int64_t)n * hwa);
  const int a = r % A;
  const float* an = anchors + (abase + r) * 4;
  const int64_t prow = (int64_t)p.row_off[seg] + (int64_t)n * p.H[seg] * p.W[seg] + r / A;
  const T* rc = rel + prow * ld + a * 4;
  const float ty = to_f<T>(rc[0]), tx = to_f<T>(rc[1]), th = to_f<T>(rc[2]), tw = to_f<T>(rc[3]);
  const float ycenter_a = (an[2] + an[0]) / 2.0f, xcenter_a = (an[3] + an[1]) / 2.0f;
  const float ha = an[2] - an[0], wa = an[3] - an[1];
  const float w = expf(tw) * wa;
  const float h = expf(th) * ha;
  const float yc = ty * ha + ycenter_a;
  const float xc = tx * wa + xcenter_a;
  float* o = out + (prow * A + a) * 4;
  o[0] = yc - h / 2.0f;
  o[1] = xc - w / 2.0f;
  o[2] = yc + h / 2.0f;
  o[3] = xc + w / 2.0f;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_anchor_boxes(int fh, int fw, float start_y, float delta_y, float start_x,
                      float delta_x, int A, const float* half_yx, float* out,
                      edet_stream_t stream) {
  EDET_REQUIRE(half_yx && out && fh > 0 && fw > 0 && A > 0, "anchor_boxes: bad argument");
  const int n = fh * fw * A;
  hipLaunchKernelGGL(k_anchor_boxes, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fh, fw, start_y,
                     delta_y, start_x, delta_x, A, half_yx, out);
  return check_launch("edet anchor_boxes");
}

int edet_generate_targets(const float* anchors, const edet_pyramid* p, int A,
                          const float* gt, const int32_t* gt_cls, const int32_t* n_gt,
                          int max_gt, float iou_thr, float* box_t, int32_t* cls_t,
                          uint8_t* mask, edet_stream_t stream) {
  EDET_REQUIRE(anchors && p && gt && gt_cls && n_gt && box_t && cls_t && mask && max_gt >= 1,
               "generate_targets: bad argument");
  int64_t total = 0;
  for (int s = 0; s < p->nseg; ++s) total += (int64_t)p->batch * p->H[s] * p->W[s] * A;
  if (total == 0) return EDET_OK;
  hipLaunchKernelGGL(k_targets, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     anchors, *p, A, gt, gt_cls, n_gt, max_gt, iou_thr, box_t, cls_t, mask, total);
  return check_launch("edet generate_targets");
}

int edet_decode_boxes(int dtype, const float* anchors, const edet_pyramid* p, int A,
                      const void* rel, int ld, float* out, edet_stream_t stream) {
  EDET_REQUIRE(anchors && p && rel && out && ld >= 4 * A, "decode_boxes: bad argument");
  int64_t total = 0;
  for (int s = 0; s < p->nseg; ++s) total += (int64_t)p->batch * p->H[s] * p->W[s] * A;
  if (total == 0) return EDET_OK;
  EDET_DTYPE_DISPATCH(dtype, T, {
    hipLaunchKernelGGL(k_decode<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       anchors, *p, A, (const T*)rel, ld, out, total);
    return check_launch("edet decode_boxes");
  });
}

}  // extern "C"
