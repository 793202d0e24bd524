// Anchor generation, training-target encoding and box decoding — the index/IoU work of
// efficientnet/utils/anchors.py.  Bit-exact with the reference's fp32 op sequence: no FMA
// contraction, correctly rounded division, argmax ties to the first index.
//
//   anchor boxes : Anchors._generate_boxes (anchors.py:47-84).  Centres follow tf.range's
//                  fp32 accumulation (start, start+delta, ...), box = centre -/+ fp32(half)
//   targets      : Anchors.generate_targets (anchors.py:91-138) with get_iou 'iou'
//                  (iou.py:27-69) and _boxes_encoder (anchors.py:219-243)
//   decode       : Anchors._boxes_decoder (anchors.py:245-274)
//   detect / NMS : Anchors.convert_outputs_one (anchors.py:161-202) with get_nms DIoU
//                  (nms.py:5-61) and get_iou 'diou' (iou.py:27-100)
#pragma clang fp contract(off)
#include <math.h>
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

// DIoU of b1 (the kept box) and b2 in get_iou's op order: iou - |c2 - c1|^2 / diag^2 with
// the norms taken as sqrt(sum of squares) and squared again, divide_no_nan for both ratios
__device__ __forceinline__ float diou_tf(const float* b1, const float* b2) {
  const float iou = iou_tf(b1, b2);
  const float eymin = fminf(b1[0], b2[0]), exmin = fminf(b1[1], b2[1]);
  const float eymax = fmaxf(b1[2], b2[2]), exmax = fmaxf(b1[3], b2[3]);
  const float c1y = (b1[0] + b1[2]) / 2.0f, c1x = (b1[1] + b1[3]) / 2.0f;
  const float c2y = (b2[0] + b2[2]) / 2.0f, c2x = (b2[1] + b2[3]) / 2.0f;
  const float dy = c2y - c1y, dx = c2x - c1x;
  const float e = sqrtf(dy * dy + dx * dx);
  const float ey = eymax - eymin, ex = exmax - exmin;
  const float d = sqrtf(ey * ey + ex * ex);
  const float e2 = e * e, d2 = d * d;
  return iou - ((d2 == 0.f) ? 0.f : e2 / d2);
}

// flat candidate index within one image (levels concatenated, each [H][W][A]) -> pyramid row
// and anchor
__device__ __forceinline__ void cand_locate(const edet_pyramid& p, int A, int n, int i, int64_t& row, int& a) {
  int seg = 0, r = i;
  for (; seg < p.nseg - 1; ++seg) {
    const int cnt = p.H[seg] * p.W[seg] * A;
    if (r < cnt) break;
    r -= cnt;
  }
  a = r % A;
  row = (int64_t)p.row_off[seg] + (int64_t)n * p.H[seg] * p.W[seg] + r / A;
}

// One block per image.  Candidates: anchors whose first-argmax class (over the NC logits) is
// not the background class 0 and whose max logit is >= score_thr (the reference stops its
// loop at the first top score below the threshold, so lower ones are never reached).
// Greedy DIoU-NMS as <= max_out rounds of {block argmax (score desc, flat index asc = the
// order of a stable descending sort), keep, suppress every live candidate with DIoU >=
// iou_thr}: the same boxes, in the same order, as the reference's sort + boolean_mask loop.
template <typename T>
__global__ __launch_bounds__(1024) void k_nms(const float* boxes, const T* cls, int ldc, edet_pyramid p, int A,
                                              int NC, int N, int max_out, float iou_thr, float score_thr,
                                              float* key, int32_t* cid, float* out_boxes, int32_t* out_cls,
                                              float* out_scores, int32_t* out_count) {
  __shared__ float wv[32];
  __shared__ int wi[32];
  __shared__ float selb[4];
  __shared__ int sel_s;
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  float* kb = key + (size_t)n * N;
  int32_t* cb = cid + (size_t)n * N;
  for (int i = tid; i < N; i += blockDim.x) {
    int64_t row;
    int a;
    cand_locate(p, A, n, i, row, a);
    const T* lg = cls + row * ldc + (int64_t)a * NC;
    int best = 0;
    float bv = to_f<T>(lg[0]);
    for (int c = 1; c < NC; ++c) {
      const float v = to_f<T>(lg[c]);
      if (v > bv) { bv = v; best = c; }  // tf.math.argmax: first maximal index
    }
    kb[i] = (best != 0 && bv >= score_thr) ? bv : -INFINITY;
    cb[i] = best;
  }
  __syncthreads();
  int count = 0;
  for (int k = 0; k < max_out; ++k) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < N; i += blockDim.x) {  // increasing i per thread: '>' keeps the lowest index
      const float v = kb[i];
      if (v > bv) { bv = v; bi = i; }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { wv[wave] = bv; wi[wave] = bi; }
    __syncthreads();
    if (tid == 0) {
      float v = wv[0];
      int id = wi[0];
      for (int w = 1; w < nw; ++w)
        if (wv[w] > v || (wv[w] == v && wi[w] < id)) { v = wv[w]; id = wi[w]; }
      sel_s = (v == -INFINITY) ? -1 : id;
      if (sel_s >= 0) {
        int64_t row;
        int a;
        cand_locate(p, A, n, id, row, a);
        const float* bx = boxes + (row * A + a) * 4;
        float* ob = out_boxes + ((size_t)n * max_out + k) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) { selb[j] = bx[j]; ob[j] = bx[j]; }
        out_cls[(size_t)n * max_out + k] = cb[id];
        out_scores[(size_t)n * max_out + k] = 1.0f / (1.0f + expf(-v));
        kb[id] = -INFINITY;
      }
    }
    __syncthreads();
    if (sel_s < 0) break;
    ++count;
    for (int i = tid; i < N; i += blockDim.x) {
      if (kb[i] == -INFINITY) continue;
      int64_t row;
      int a;
      cand_locate(p, A, n, i, row, a);
      if (diou_tf(selb, boxes + (row * A + a) * 4) >= iou_thr) kb[i] = -INFINITY;
    }
    __syncthreads();
  }
  if (tid == 0) out_count[n] = count;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_detect_nms(int dtype, const float* boxes, const void* cls, int ldc, const edet_pyramid* p, int A,
                    int NC, int max_out, float iou_thr, float score_thr, void* scratch,
                    float* out_boxes, int32_t* out_cls, float* out_scores, int32_t* out_count,
                    edet_stream_t stream) {
  EDET_REQUIRE(boxes && cls && p && scratch && out_boxes && out_cls && out_scores && out_count,
               "detect_nms: null argument");
  EDET_REQUIRE(A > 0 && NC > 0 && ldc >= A * NC && max_out > 0, "detect_nms: bad sizes");
  int N = 0;
  for (int s = 0; s < p->nseg; ++s) N += p->H[s] * p->W[s] * A;
  if (p->batch == 0 || N == 0) return EDET_OK;
  float* key = (float*)scratch;
  int32_t* cid = (int32_t*)(key + (size_t)p->batch * N);
  EDET_DTYPE_DISPATCH(dtype, T, {
    EDET_LAUNCH(k_nms<T>, dim3(p->batch), dim3(1024), 0, (hipStream_t)stream, boxes, (const T*)cls, ldc, *p,
                       A, NC, N, max_out, iou_thr, score_thr, key, cid, out_boxes, out_cls, out_scores, out_count);
    return check_launch("edet detect_nms");
  });
}

int edet_anchor_boxes(int fh, int fw, float start_y, float delta_y, float start_x,
                      float delta_x, int A, const float* half_yx, float* out,
                      edet_stream_t stream) {
  EDET_REQUIRE(half_yx && out && fh > 0 && fw > 0 && A > 0, "anchor_boxes: bad argument");
  const int n = fh * fw * A;
  EDET_LAUNCH(k_anchor_boxes, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, fh, fw, start_y,
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
  EDET_LAUNCH(k_targets, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
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
    EDET_LAUNCH(k_decode<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       anchors, *p, A, (const T*)rel, ld, out, total);
    return check_launch("edet decode_boxes");
  });
}

}  // extern "C"
