// Detection loss: sigmoid focal loss (losses/focal_loss.py:26-52) + Huber box loss
// (losses/box_loss.py:21-30) summed as in EfficientDetNetTrain._get_loss
// (efficientnet/efficientdet_net_train.py:41-52), forward and backward in one pass.
//
// Per level l (segment of the pyramid), with N+ = sum(masks) + 1 over the batch:
//   focal_l = sum FL / (N+ * B*H_l*W_l*A*NC)      (FL / normalizer, then Keras
//                                                  SUM_OVER_BATCH_SIZE = mean over elements)
//   box_l   = sum huber(pred - t) * [t != 0] / (4 N+)
//   loss   += box_weight * box_l + focal_l
// The one-hot class target of the reference (anchors.py:133) is represented by its index.
#include "common.hpp"

namespace edet {

constexpr int LCLS_ROWS = 32;  // rows per classification block (8 / 16 / 32 / 64: 363 / 197 / 191 / 200 us)
constexpr int LBOX_ROWS = 256;

struct LossArgs {
  const void* cls;
  const void* box;
  const int32_t* cls_t;
  const float* box_t;
  const float* npos;
  void* dcls;
  void* dbox;
  float* loss;
  float* parts;
  edet_pyramid p;
  int ldc, ldb, A, NC;
  float alpha, gamma, delta, box_weight, count_scale;
  int nb_cls;
};

__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// focal loss value and d/dx for one logit (focal_loss.py:42-52, TF sigmoid CE formulation)
__device__ __forceinline__ void focal_elem(float x, float y, float alpha, float gamma, bool g15, float& fl, float& dfl) {
  // v_rcp_f32 / v_sqrt_f32 (1 ulp) instead of the correctly rounded division and square root
  // the build flags select for '/' and sqrtf: this kernel is VALU-bound over 127 M logits
  const float z = __expf(-fabsf(x));
  const float r = __builtin_amdgcn_rcpf(1.f + z);
  const float p = x >= 0.f ? r : z * r;                  // sigmoid(x)
  const float pt = y * p + (1.f - y) * (1.f - p);
  const float at = y * alpha + (1.f - y) * (1.f - alpha);
  const float om = fmaxf(1.f - pt, 0.f);
  float mod, dmodf;                                      // (1-pt)^g and g*(1-pt)^(g-1)
  if (g15) {
    const float sq = __builtin_amdgcn_sqrtf(om);
    mod = om * sq;
    dmodf = 1.5f * sq;
  } else {
    const float lg = __logf(om);
    mod = om > 0.f ? __expf(gamma * lg) : 0.f;
    dmodf = om > 0.f ? gamma * __expf((gamma - 1.f) * lg) : 0.f;
  }
  const float ce = fmaxf(x, 0.f) - x * y + __logf(1.f + z);
  const float dpt = (2.f * y - 1.f) * p * (1.f - p);
  fl = at * mod * ce;
  dfl = at * (-dmodf * dpt * ce + mod * (p - y));
}

// gamma = 1.5 with a 0/1 target, branch-free and cancellation-free (same value as focal_elem):
// with z = exp(-|x|), r = 1/(1+z): sigmoid = x >= 0 ? r : z r, and
//   q  = 1 - pt = (x >= 0) != y ? r : z r           (the modulating base, exact)
//   ce = log(1+z) + max(y ? -x : x, 0)
//   p (1-p) = z r^2,   p - y = (y ? -1 : 1) q,   dpt = -(y ? -1 : 1) p (1-p)
//   fl  = at q^1.5 ce
//   dfl = at (y ? -1 : 1) sqrt(q) (1.5 p (1-p) ce + q^2)
// kpos / kneg fold at * sign * (1 / normaliser) for y = 1 / y = 0.
// Three transcendentals per logit instead of four (round 6): with h = exp(-|x|/2) and
// s = rsqrt(1 + h^2), z = h^2, r = s^2, sqrt(r) = s, sqrt(z r) = h s and log(1+z) = -2 log(s),
// so the sigmoid's reciprocal and the modulating square root come from one v_rsq_f32
__device__ __forceinline__ void focal_elem15(float x, bool y, float apos, float aneg, float kpos, float kneg,
                                             float& fl, float& dfl) {
  const float h = __builtin_amdgcn_exp2f(fabsf(x) * -0.72134752044448170f);  // exp(-|x|/2)
  const float z = h * h;
  const float s = __builtin_amdgcn_rsqf(1.f + z);
  const float r = s * s;
  const float zr = z * r;
  const bool flip = (x >= 0.f) != y;
  const float q = flip ? r : zr;
  const float sq = flip ? s : h * s;
  const float ce = fmaf(-1.3862943611198906f, __builtin_amdgcn_logf(s), fmaxf(y ? -x : x, 0.f));
  fl = (y ? apos : aneg) * q * sq * ce;
  dfl = (y ? kpos : kneg) * sq * fmaf(1.5f * zr * r, ce, q * q);
}

// Two logits at a time in packed fp32 (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: the
// multiplies of focal_elem15 on both lanes of a pair in one instruction; the transcendentals and
// selects stay scalar).  Same formula as focal_elem15.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void focal_pair15(f2v x, bool y0, bool y1, float apos, float aneg, float kpos, float kneg,
                                             f2v& fl, f2v& dfl) {
  const f2v t = f2v{fabsf(x.x), fabsf(x.y)} * -0.72134752044448170f;
  const f2v h = f2v{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  const f2v z = h * h;
  const f2v z1 = z + 1.f;
  const f2v sv = f2v{__builtin_amdgcn_rsqf(z1.x), __builtin_amdgcn_rsqf(z1.y)};
  const f2v r = sv * sv;
  const f2v zr = z * r;
  const f2v hs = h * sv;
  const bool fl0 = (x.x >= 0.f) != y0, fl1 = (x.y >= 0.f) != y1;
  const f2v q = f2v{fl0 ? r.x : zr.x, fl1 ? r.y : zr.y};
  const f2v sq = f2v{fl0 ? sv.x : hs.x, fl1 ? sv.y : hs.y};
  const f2v lg = f2v{__builtin_amdgcn_logf(sv.x), __builtin_amdgcn_logf(sv.y)};
  const f2v mx = f2v{fmaxf(y0 ? -x.x : x.x, 0.f), fmaxf(y1 ? -x.y : x.y, 0.f)};
  const f2v ce = lg * -1.3862943611198906f + mx;
  const f2v a = f2v{y0 ? apos : aneg, y1 ? apos : aneg};
  const f2v k = f2v{y0 ? kpos : kneg, y1 ? kpos : kneg};
  fl = a * q * sq * ce;
  dfl = k * sq * ((zr * r * 1.5f) * ce + q * q);
}

template <typename T>
__global__ __launch_bounds__(256) void k_loss(LossArgs g) {
  __shared__ float red[4];
  const int tid = threadIdx.x;
  const float npos = *g.npos + 1.f;
  const bool g15 = g.gamma == 1.5f;
  int b = blockIdx.x;
  if (b < g.nb_cls) {
    int seg, chunk;
    chunk_lookup(g.p, LCLS_ROWS, b, seg, chunk);
    const int rows = seg_rows(g.p, seg);
    const int m0 = g.p.row_off[seg] + chunk * LCLS_ROWS;
    const int nr = min(LCLS_ROWS, g.p.row_off[seg] + rows - m0);
    const int AN = g.A * g.NC;
    const float inv = 1.f / (npos * (float)rows * (float)AN * g.count_scale);
    T* X = (T*)g.cls;  // logits; gradient written in place when dcls == cls
    T* D = (T*)g.dcls;
    float s = 0.f;
    if (g15 && g.NC >= 8 && (g.ldc & 7) == 0 && D == X && sizeof(T) == 2) {
      // the training path (gamma = 1.5, bf16 logits, gradient in place): the thread's vectors
      // walked incrementally (no division per vector), a vector's positives as two column
      // indices (NC >= 8: it spans at most two anchors), the logits in packed pairs
      const int nvec = g.ldc / 8, step_r = 256 / nvec, step_v = 256 - step_r * nvec;
      const float invNC = 1.f / (float)g.NC;
      const float apos = g.alpha, aneg = 1.f - g.alpha, kpos = -g.alpha * inv, kneg = (1.f - g.alpha) * inv;
      int r = tid / nvec, vi = tid - r * nvec;
      while (r < nr) {
        const int cv = vi * 8, m = m0 + r;
        T* px = X + (size_t)m * g.ldc + cv;
        float x[8], d[8];
        ld8(px, x);
        const int32_t* tr = g.cls_t + (size_t)m * g.A;
        const int a0 = (int)(((float)cv + 0.5f) * invNC);  // exact for cv < 2^20
        const int ta = tr[a0], tb = (a0 + 1 < g.A) ? tr[a0 + 1] : -1;
        const int p0 = (ta >= 0 && ta < g.NC) ? a0 * g.NC + ta : -1;
        const int p1 = (tb >= 0 && tb < g.NC) ? (a0 + 1) * g.NC + tb : -1;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int c0 = cv + j, c1 = c0 + 1;
          f2v fl, dfl;
          focal_pair15(f2v{x[j], x[j + 1]}, c0 == p0 || c0 == p1, c1 == p0 || c1 == p1, apos, aneg, kpos, kneg,
                       fl, dfl);
          const bool v0 = c0 < AN, v1 = c1 < AN;
          d[j] = v0 ? dfl.x : 0.f;
          d[j + 1] = v1 ? dfl.y : 0.f;
          s += (v0 ? fl.x : 0.f) + (v1 ? fl.y : 0.f);
        }
        st8(px, d);
        // next vector of this thread (256 further): no division per vector
        vi += step_v;
        r += step_r;
        if (vi >= nvec) { vi -= nvec; ++r; }
      }
      // (two vectors in flight per trip measured the same, r06ab: 166.8 -> 162.1 us against
      // 160.8 -> 156.9 for this form, r06aa)
    } else if ((g.ldc & 7) == 0 && (!D || D == X)) {
      const int nvec = g.ldc / 8;
      for (int e = tid; e < nr * nvec; e += 256) {
        const int r = e / nvec, cv = (e - r * nvec) * 8;
        const int m = m0 + r;
        T* px = X + (size_t)m * g.ldc + cv;
        float x[8], d[8];
        ld8(px, x);
        const int32_t* tr = g.cls_t + (size_t)m * g.A;
        // (anchor, class) of the vector's first column; the next 7 step without a division
        // and, with NC >= 8, stay within two anchors whose targets are read once
        const int a0 = cv / g.NC;
        int a = a0, c = cv - a0 * g.NC;
        const int ta = tr[a0], tb = (a0 + 1 < g.A) ? tr[a0 + 1] : -1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int col = cv + j;
          d[j] = 0.f;
          if (j > 0 && ++c == g.NC) { c = 0; ++a; }
          if (col < AN) {
            const bool yb = (g.NC >= 8 ? (a == a0 ? ta : tb) : tr[a]) == c;
            float fl, dfl;
            if (g15) {
              focal_elem15(x[j], yb, g.alpha, 1.f - g.alpha, -g.alpha * inv, (1.f - g.alpha) * inv, fl, dfl);
              d[j] = dfl;
            } else {
              focal_elem(x[j], yb ? 1.f : 0.f, g.alpha, g.gamma, g15, fl, dfl);
              d[j] = dfl * inv;
            }
            s += fl;
          }
        }
        if (D) st8(px, d);
      }
    } else {  // generic strides / separate gradient buffer
      for (int e = tid; e < nr * AN; e += 256) {
        const int r = e / AN, col = e - r * AN;
        const int m = m0 + r;
        const int a = col / g.NC, c = col - a * g.NC;
        const float x = to_f<T>(X[(size_t)m * g.ldc + col]);
        const float y = (g.cls_t[(size_t)m * g.A + a] == c) ? 1.f : 0.f;
        float fl, dfl;
        focal_elem(x, y, g.alpha, g.gamma, g15, fl, dfl);
        s += fl;
        if (D) D[(size_t)m * g.ldc + col] = from_f<T>(dfl * inv);
      }
      if (D && g.ldc > AN) {
        const int pad = g.ldc - AN;
        for (int e = tid; e < nr * pad; e += 256) {
          const int r = e / pad;
          D[(size_t)(m0 + r) * g.ldc + AN + (e - r * pad)] = from_f<T>(0.f);
        }
      }
    }
    s = block_sum(s, red);
    if (tid == 0) {
      atomicAdd(g.loss, s * inv);
      if (g.parts) atomicAdd(g.parts + seg, s * inv);
    }
    return;
  }
  b -= g.nb_cls;
  int seg, chunk;
  chunk_lookup(g.p, LBOX_ROWS, b, seg, chunk);
  const int rows = seg_rows(g.p, seg);
  const int m0 = g.p.row_off[seg] + chunk * LBOX_ROWS;
  const int nr = min(LBOX_ROWS, g.p.row_off[seg] + rows - m0);
  const int A4 = g.A * 4;
  const float inv = 1.f / (4.f * npos);
  T* P = (T*)g.box;
  T* D = (T*)g.dbox;
  const float dl = g.delta;
  float s = 0.f;
  for (int e = tid; e < nr * A4; e += 256) {
    const int r = e / A4, col = e - r * A4;
    const int m = m0 + r;
    const float t = g.box_t[(size_t)m * A4 + col];
    const float pr = to_f<T>(P[(size_t)m * g.ldb + col]);
    const float mask = (t != 0.f) ? 1.f : 0.f;
    const float err = pr - t, ae = fabsf(err);
    const float h = (ae <= dl) ? 0.5f * err * err : 0.5f * dl * dl + dl * (ae - dl);
    s += h * mask;
    if (D) {
      const float dh = (ae <= dl) ? err : (err > 0.f ? dl : -dl);
      D[(size_t)m * g.ldb + col] = from_f<T>(dh * mask * inv * g.box_weight);
    }
  }
  if (D && g.ldb > A4) {
    const int pad = g.ldb - A4;
    for (int e = tid; e < nr * pad; e += 256) {
      const int r = e / pad;
      D[(size_t)(m0 + r) * g.ldb + A4 + (e - r * pad)] = from_f<T>(0.f);
    }
  }
  s = block_sum(s, red);
  if (tid == 0) {
    atomicAdd(g.loss, s * inv * g.box_weight);
    if (g.parts) atomicAdd(g.parts + EDET_MAX_SEG + seg, s * inv);
  }
}

// 16 mask bytes per thread and step, few blocks: the count ends in one same-address atomic
// per block (exact: integer-valued floats far below 2^24)
__global__ void k_count_pos(const uint8_t* mask, int64_t n, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t nv = n / 16, stride = (int64_t)gridDim.x * 256;
  // four 16-byte vectors per trip, all requested before any is counted (the 64-block grid
  // walked ~6 dependent loads per thread: 14.9 us for D0's 1.6 MB of masks)
  for (int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x; i0 < nv; i0 += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * stride;
      v[u] = i < nv ? reinterpret_cast<const uint4*>(mask)[i] : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int b = 0; b < 4; ++b) s += ((w4[k] >> (8 * b)) & 0xffu) ? 1.f : 0.f;
    }
  }
  for (int64_t i = nv * 16 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += mask[i] ? 1.f : 0.f;
  s = block_sum(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

__global__ void k_onehot_index(const float* onehot, int64_t n, int NC, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* p = onehot + i * NC;
  int best = 0;
  float bv = p[0];
  for (int c = 1; c < NC; ++c)
    if (p[c] > bv) { bv = p[c]; best = c; }
  out[i] = best;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_detection_loss(int dtype, const void* cls, int ldc, const void* box, int ldb,
                        const edet_pyramid* p, int A, int NC, const int32_t* cls_t,
                        const float* box_t, const float* npos_sum, float alpha, float gamma,
                        float delta, float box_weight, float focal_count_scale, void* dcls,
                        void* dbox, float* loss, float* level_parts, edet_stream_t stream) {
  EDET_REQUIRE(cls && box && p && cls_t && box_t && npos_sum && loss, "detection_loss: null argument");
  EDET_REQUIRE(ldc >= A * NC && ldb >= A * 4 && p->nseg >= 1 && p->nseg <= EDET_MAX_SEG,
               "detection_loss: bad strides");
  LossArgs g{};
  g.cls = cls; g.box = box; g.cls_t = cls_t; g.box_t = box_t; g.npos = npos_sum; g.dcls = dcls;
  g.dbox = dbox; g.loss = loss; g.parts = level_parts; g.p = *p; g.ldc = ldc; g.ldb = ldb;
  g.A = A; g.NC = NC; g.alpha = alpha; g.gamma = gamma; g.delta = delta; g.box_weight = box_weight;
  g.count_scale = focal_count_scale > 0.f ? focal_count_scale : 1.f;
  g.nb_cls = total_chunks(*p, LCLS_ROWS);
  const int nb = g.nb_cls + total_chunks(*p, LBOX_ROWS);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_loss<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, g);
    return check_launch("edet detection_loss");
  });
}

int edet_count_positives(const uint8_t* mask, int64_t n, float* out, edet_stream_t stream) {
  EDET_REQUIRE(mask && out, "count_positives: null argument");
  if (n <= 0) return EDET_OK;
  EDET_REQUIRE(((uintptr_t)mask & 15) == 0, "count_positives: mask must be 16-byte aligned");
  // one trip of four vectors per thread where that takes at most 128 blocks (each block ends
  // in one fp32 atomic on the same address: integer counts, exact in any order)
  int nb = (int)((n / 16 + 1023) / 1024);
  if (nb > 128) nb = 128;
  if (nb < 1) nb = 1;
  EDET_LAUNCH(k_count_pos, dim3(nb), dim3(256), 0, (hipStream_t)stream, mask, n, out);
  return check_launch("edet count_positives");
}

int edet_onehot_to_index(const float* onehot, int64_t n, int NC, int32_t* out,
                         edet_stream_t stream) {
  EDET_REQUIRE(onehot && out && NC > 0, "onehot_to_index: bad argument");
  if (n <= 0) return EDET_OK;
  EDET_LAUNCH(k_onehot_index, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     onehot, n, NC, out);
  return check_launch("edet onehot_to_index");
}

}  // extern "C"
