// Training-mode BatchNorm backward, swish', SE squeeze/excite (fwd+bwd), the heads'
// drop-connect residual, and the moving-statistics update.
//
// The forward BN never runs as its own pass: producers (conv epilogues) emit per-channel
// sum / sum-of-squares, consumers normalise while loading ("lazy" values, common.hpp).
// Backward of a lazy value v = act(bn(x)) * gate is two passes over the rows:
//   reduce : dbeta += sum du, dgamma += sum du * xhat          (du = d(bn output))
//   apply  : dx = gamma*rstd * (du - dbeta/M - xhat*dgamma/M)
// which is the TF FusedBatchNormGradV3 training formula with
// du = (dv * gate + dsq) * swish'(u) for the swish / SE cases (layers/se.py:35-39,
// layers/mb_conv_block.py:144-150).
#include "common.hpp"

namespace edet {

constexpr int RCH = 256;  // rows per chunk
constexpr int RCB = 64;   // channels per block

struct LArgs {
  edet_lazy lz;
  edet_lazy res;
  edet_pyramid p;
  edet_segout grads;
  const void* dv;
  void* dx;
  const float* dv_scale;
  const float* dsq;
  float* out;  // se_squeeze / gate_grad output [batch][C]
  int C, ncb, accumulate, hw, chunks_per_img;
};

// per-block channel table: affine (sc, sh) and (mean, rstd)
__device__ __forceinline__ void load_chan_table(const edet_lazy& lz, int seg, float inv, int c0, int C,
                                                float2* af, float2* mr) {
  const int tid = threadIdx.x;
  if (tid < RCB) {
    const int c = c0 + tid;
    float2 a = make_float2(1.f, 0.f), b = make_float2(0.f, 1.f);
    if (c < C && lz.bn.enabled) {
      a = bn_affine(lz.bn, seg, c, inv);
      b = bn_mean_rstd(lz.bn, seg, c, inv);
    }
    af[tid] = a;
    mr[tid] = b;
  }
}

// du for 8 channels of one row; also returns xhat
template <typename T>
__device__ __forceinline__ void lazy_du(const LArgs& g, int seg, int m, int n, int cv8, int cc, int nc,
                                        const float2* af, const float2* mr, float* du, float* xh) {
  float x[8], d[8];
  ld8m((const T*)g.lz.x + (size_t)m * g.lz.ld + cc, nc, x);
  ld8m((const T*)g.dv + (size_t)m * g.C + cc, nc, d);
  const float dvs = g.dv_scale ? g.dv_scale[seg * g.p.batch + n] : 1.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float2 a = af[cv8 + j];
    const float u = x[j] * a.x + a.y;
    float gg = d[j] * dvs;
    if (j < nc) {
      if (g.lz.gate) gg *= g.lz.gate[(size_t)n * g.C + cc + j];
      if (g.dsq) gg += g.dsq[(size_t)n * g.C + cc + j];
    }
    du[j] = g.lz.act ? gg * dswishf_(u) : gg;
    const float2 b = mr[cv8 + j];
    xh[j] = (x[j] - b.x) * b.y;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_lazy_bwd_reduce(LArgs g) {
  __shared__ float2 af[RCB], mr[RCB];
  __shared__ float red[2][32][RCB + 1];
  const int tid = threadIdx.x, cv = tid & 7, rs = tid >> 3;
  const int cb = blockIdx.x % g.ncb;
  int seg, chunk;
  chunk_lookup(g.p, RCH, blockIdx.x / g.ncb, seg, chunk);
  const int c0 = cb * RCB;
  const int rows = seg_rows(g.p, seg);
  load_chan_table(g.lz, seg, 1.f / (float)rows, c0, g.C, af, mr);
  __syncthreads();
  const int off = g.p.row_off[seg];
  const int m_begin = off + chunk * RCH, m_end = min(off + rows, m_begin + RCH);
  const int hw = g.p.H[seg] * g.p.W[seg];
  const int cc = c0 + cv * 8, nc = g.C - cc;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
  if (nc > 0) {
    for (int m = m_begin + rs; m < m_end; m += 32) {
      const int n = (m - off) / hw;
      float du[8], xh[8];
      lazy_du<T>(g, seg, m, n, cv * 8, cc, nc, af, mr, du, xh);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s[j] += du[j]; q[j] += du[j] * xh[j]; }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[0][rs][cv * 8 + j] = s[j]; red[1][rs][cv * 8 + j] = q[j]; }
  __syncthreads();
  if (tid < RCB && c0 + tid < g.C) {
    float ss = 0.f, qq = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) { ss += red[0][i][tid]; qq += red[1][i][tid]; }
    atomicAdd(g.grads.b[seg] + c0 + tid, ss);  // dbeta
    atomicAdd(g.grads.a[seg] + c0 + tid, qq);  // dgamma
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_lazy_bwd_apply(LArgs g) {
  __shared__ float2 af[RCB], mr[RCB], gb[RCB];
  const int tid = threadIdx.x, cv = tid & 7, rs = tid >> 3;
  const int cb = blockIdx.x % g.ncb;
  int seg, chunk;
  chunk_lookup(g.p, RCH, blockIdx.x / g.ncb, seg, chunk);
  const int c0 = cb * RCB;
  const int rows = seg_rows(g.p, seg);
  const float inv = 1.f / (float)rows;
  load_chan_table(g.lz, seg, inv, c0, g.C, af, mr);
  if (tid < RCB) {
    const int c = c0 + tid;
    gb[tid] = (g.lz.bn.enabled && c < g.C) ? make_float2(g.grads.a[seg][c] * inv, g.grads.b[seg][c] * inv)
                                          : make_float2(0.f, 0.f);
  }
  __syncthreads();
  const int off = g.p.row_off[seg];
  const int m_begin = off + chunk * RCH, m_end = min(off + rows, m_begin + RCH);
  const int hw = g.p.H[seg] * g.p.W[seg];
  const int cc = c0 + cv * 8, nc = g.C - cc;
  if (nc <= 0) return;
  T* DX = (T*)g.dx;
  for (int m = m_begin + rs; m < m_end; m += 32) {
    const int n = (m - off) / hw;
    float du[8], xh[8], o[8];
    lazy_du<T>(g, seg, m, n, cv * 8, cc, nc, af, mr, du, xh);
    if (g.lz.bn.enabled) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 d = gb[cv * 8 + j];  // (dgamma/M, dbeta/M)
        o[j] = af[cv * 8 + j].x * (du[j] - d.y - xh[j] * d.x);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = du[j];
    }
    acc8m(DX + (size_t)m * g.C + cc, nc, o, g.accumulate);
  }
}

// out[n][c] += (scale) * sum_hw f(row)   -- SE squeeze (mean of v(x)) or gate grad (dv * v(x))
template <typename T, bool GATEGRAD>
__global__ __launch_bounds__(256) void k_img_reduce(LArgs g) {
  __shared__ float2 af[RCB], mr[RCB];
  __shared__ float red[32][RCB + 1];
  const int tid = threadIdx.x, cv = tid & 7, rs = tid >> 3;
  const int cb = blockIdx.x % g.ncb;
  const int id = blockIdx.x / g.ncb;
  const int n = id / g.chunks_per_img, chunk = id - n * g.chunks_per_img;
  const int c0 = cb * RCB;
  const int rows = seg_rows(g.p, 0);
  load_chan_table(g.lz, 0, 1.f / (float)rows, c0, g.C, af, mr);
  __syncthreads();
  const int m_begin = n * g.hw + chunk * RCH, m_end = min((n + 1) * g.hw, m_begin + RCH);
  const int cc = c0 + cv * 8, nc = g.C - cc;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (nc > 0) {
    for (int m = m_begin + rs; m < m_end; m += 32) {
      float x[8];
      ld8m((const T*)g.lz.x + (size_t)m * g.lz.ld + cc, nc, x);
      float d[8];
      if (GATEGRAD) ld8m((const T*)g.dv + (size_t)m * g.C + cc, nc, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = lazy_apply(x[j], af[cv * 8 + j], g.lz.act);
        s[j] += GATEGRAD ? d[j] * v : v;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rs][cv * 8 + j] = s[j];
  __syncthreads();
  if (tid < RCB && c0 + tid < g.C) {
    float ss = 0.f;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) ss += red[i][tid];
    if (!GATEGRAD) ss *= 1.f / (float)g.hw;
    atomicAdd(g.out + (size_t)n * g.C + c0 + tid, ss);
  }
}

// SE excite: z1 = W1 s + b1 ; gate = sigmoid(W2 swish(z1) + b2)   (layers/se.py:36-39)
__global__ __launch_bounds__(256) void k_se_fwd(int C, int R, const float* s, const float* w1,
                                                const float* b1, const float* w2, const float* b2,
                                                float* z1, float* gate) {
  extern __shared__ float sh[];
  float* ss = sh;       // [C]
  float* s1 = sh + C;   // [R]
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < C; c += 256) ss[c] = s[(size_t)n * C + c];
  __syncthreads();
  for (int r = wave; r < R; r += 4) {
    float a = 0.f;
    for (int c = lane; c < C; c += 64) a += w1[(size_t)r * C + c] * ss[c];
    a = wave_sum(a);
    if (lane == 0) {
      const float z = a + b1[r];
      z1[(size_t)n * R + r] = z;
      s1[r] = z / (1.f + expf(-z));
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float a = b2[c];
    for (int r = 0; r < R; ++r) a += w2[(size_t)c * R + r] * s1[r];
    gate[(size_t)n * C + c] = 1.f / (1.f + expf(-a));
  }
}

__global__ __launch_bounds__(256) void k_se_bwd(int C, int R, int HW, const float* s, const float* z1,
                                                const float* gate, const float* dgate, const float* w1,
                                                const float* w2, float* dw1, float* db1, float* dw2,
                                                float* db2, float* dsq) {
  extern __shared__ float sh[];
  float* ss = sh;            // [C] squeeze input
  float* dz2 = sh + C;       // [C]
  float* s1 = sh + 2 * C;    // [R]
  float* dz1 = s1 + R;       // [R]
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int c = tid; c < C; c += 256) {
    ss[c] = s[(size_t)n * C + c];
    const float gv = gate[(size_t)n * C + c];
    const float d = dgate[(size_t)n * C + c] * gv * (1.f - gv);
    dz2[c] = d;
    atomicAdd(db2 + c, d);
  }
  for (int r = tid; r < R; r += 256) {
    const float z = z1[(size_t)n * R + r];
    s1[r] = z / (1.f + expf(-z));
  }
  __syncthreads();
  for (int e = tid; e < C * R; e += 256) {
    const int c = e / R, r = e - c * R;
    atomicAdd(dw2 + e, dz2[c] * s1[r]);
  }
  for (int r = wave; r < R; r += 4) {
    float a = 0.f;
    for (int c = lane; c < C; c += 64) a += dz2[c] * w2[(size_t)c * R + r];
    a = wave_sum(a);
    if (lane == 0) {
      const float z = z1[(size_t)n * R + r];
      const float sg = 1.f / (1.f + expf(-z));
      const float d = a * sg * (1.f + z * (1.f - sg));
      dz1[r] = d;
      atomicAdd(db1 + r, d);
    }
  }
  __syncthreads();
  for (int e = tid; e < R * C; e += 256) {
    const int r = e / C, c = e - r * C;
    atomicAdd(dw1 + e, dz1[r] * ss[c]);
  }
  const float inv_hw = 1.f / (float)HW;
  for (int c = tid; c < C; c += 256) {
    float a = 0.f;
    for (int r = 0; r < R; ++r) a += dz1[r] * w1[(size_t)r * C + c];
    dsq[(size_t)n * C + c] = a * inv_hw;
  }
}

// heads: out = v(x) * scale[seg][n] + v(res)   (class_net.py:93-96 with drop_connect.py:4-18)
template <typename T>
__global__ __launch_bounds__(256) void k_residual(LArgs g) {
  __shared__ float2 ax[RCB], ar[RCB], dummy[RCB];
  const int tid = threadIdx.x, cv = tid & 7, rs = tid >> 3;
  const int cb = blockIdx.x % g.ncb;
  int seg, chunk;
  chunk_lookup(g.p, RCH, blockIdx.x / g.ncb, seg, chunk);
  const int c0 = cb * RCB;
  const int rows = seg_rows(g.p, seg);
  const float inv = 1.f / (float)rows;
  load_chan_table(g.lz, seg, inv, c0, g.C, ax, dummy);
  __syncthreads();
  load_chan_table(g.res, seg, inv, c0, g.C, ar, dummy);
  __syncthreads();
  const int off = g.p.row_off[seg];
  const int m_begin = off + chunk * RCH, m_end = min(off + rows, m_begin + RCH);
  const int hw = g.p.H[seg] * g.p.W[seg];
  const int cc = c0 + cv * 8, nc = g.C - cc;
  if (nc <= 0) return;
  T* OUT = (T*)g.dx;
  for (int m = m_begin + rs; m < m_end; m += 32) {
    const int n = (m - off) / hw;
    const float sc = g.dv_scale ? g.dv_scale[seg * g.p.batch + n] : 1.f;
    float x[8], r[8], o[8];
    ld8m((const T*)g.lz.x + (size_t)m * g.lz.ld + cc, nc, x);
    ld8m((const T*)g.res.x + (size_t)m * g.res.ld + cc, nc, r);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = lazy_apply(x[j], ax[cv * 8 + j], g.lz.act) * sc + lazy_apply(r[j], ar[cv * 8 + j], g.res.act);
    st8m(OUT + (size_t)m * g.C + cc, nc, o);
  }
}

// Keras BatchNormalization moving statistics: m -= (m - batch) * (1 - momentum), with the
// Bessel-corrected batch variance that FusedBatchNormV3 returns in training mode.
__global__ void k_bn_update(int64_t n, const float* sum, const float* sq, const float* count,
                            float momentum, float* mmean, float* mvar) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float cnt = count[i];
  const float mean = sum[i] / cnt;
  const float var = fmaxf(sq[i] / cnt - mean * mean, 0.f);
  const float unb = var * cnt / fmaxf(cnt - 1.f, 1.f);
  mmean[i] -= (mmean[i] - mean) * (1.f - momentum);
  mvar[i] -= (mvar[i] - unb) * (1.f - momentum);
}

__global__ void k_bn_infer_stats(int64_t n, const float* mm, const float* mv, const float* count, float* sum,
                                 float* sq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float c = count[i], m = mm[i];
  sum[i] = m * c;
  sq[i] = (mv[i] + m * m) * c;
}

static int lazy_checks(const edet_lazy* x, const edet_pyramid* p, int C) {
  EDET_REQUIRE(x && p && x->x, "lazy: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0, "lazy: need C%%8==0, ld%%8==0 (C=%d ld=%d)", C, x->ld);
  EDET_REQUIRE(p->nseg >= 1 && p->nseg <= EDET_MAX_SEG, "lazy: bad pyramid");
  EDET_REQUIRE(x->gate == nullptr || p->nseg == 1, "lazy: gate needs one segment");
  return EDET_OK;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_lazy_bwd_reduce(int dtype, const edet_lazy* x, const edet_pyramid* p, int C,
                         const void* dv, const float* dv_scale, const float* dsq,
                         const edet_segout* grads, edet_stream_t stream) {
  int rc = lazy_checks(x, p, C);
  if (rc) return rc;
  EDET_REQUIRE(dv && grads && x->bn.enabled, "lazy_bwd_reduce: needs dv, grads and an enabled BN");
  EDET_REQUIRE(dsq == nullptr || p->nseg == 1, "lazy_bwd_reduce: dsq needs one segment");
  LArgs g{};
  g.lz = *x; g.p = *p; g.grads = *grads; g.dv = dv; g.dv_scale = dv_scale; g.dsq = dsq; g.C = C;
  g.ncb = cdiv(C, RCB);
  const int nb = total_chunks(*p, RCH) * g.ncb;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) hipLaunchKernelGGL(k_lazy_bwd_reduce<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, g);
    return check_launch("edet lazy_bwd_reduce");
  });
}

int edet_lazy_bwd_apply(int dtype, const edet_lazy* x, const edet_pyramid* p, int C,
                        const void* dv, const float* dv_scale, const float* dsq,
                        const edet_segout* grads, void* dx, int accumulate,
                        edet_stream_t stream) {
  int rc = lazy_checks(x, p, C);
  if (rc) return rc;
  EDET_REQUIRE(dv && dx, "lazy_bwd_apply: null dv/dx");
  EDET_REQUIRE(!x->bn.enabled || grads, "lazy_bwd_apply: BN needs the reduced grads");
  EDET_REQUIRE(dsq == nullptr || p->nseg == 1, "lazy_bwd_apply: dsq needs one segment");
  LArgs g{};
  g.lz = *x; g.p = *p; if (grads) g.grads = *grads; g.dv = dv; g.dx = dx; g.dv_scale = dv_scale;
  g.dsq = dsq; g.C = C; g.accumulate = accumulate;
  g.ncb = cdiv(C, RCB);
  const int nb = total_chunks(*p, RCH) * g.ncb;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) hipLaunchKernelGGL(k_lazy_bwd_apply<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, g);
    return check_launch("edet lazy_bwd_apply");
  });
}

static int img_reduce(int dtype, bool gategrad, const edet_lazy* x, int B, int HW, int C,
                      const void* dv, float* out, hipStream_t s) {
  EDET_REQUIRE(x && out && x->x && (!gategrad || dv), "se reduce: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0, "se reduce: need C%%8==0");
  LArgs g{};
  g.lz = *x; g.lz.gate = nullptr;  // the pre-gate value
  g.p.nseg = 1; g.p.batch = B; g.p.row_off[0] = 0; g.p.H[0] = HW; g.p.W[0] = 1;
  g.dv = dv; g.out = out; g.C = C; g.hw = HW;
  g.ncb = cdiv(C, RCB);
  g.chunks_per_img = cdiv(HW, RCH);
  const int nb = B * g.chunks_per_img * g.ncb;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (gategrad) hipLaunchKernelGGL((k_img_reduce<T, true>), dim3(nb), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_img_reduce<T, false>), dim3(nb), dim3(256), 0, s, g);
    return check_launch("edet se reduce");
  });
}

int edet_se_squeeze(int dtype, const edet_lazy* x, int B, int HW, int C, float* s,
                    edet_stream_t stream) {
  return img_reduce(dtype, false, x, B, HW, C, nullptr, s, (hipStream_t)stream);
}

int edet_gate_grad(int dtype, const edet_lazy* x, int B, int HW, int C, const void* dv,
                   float* dgate, edet_stream_t stream) {
  return img_reduce(dtype, true, x, B, HW, C, dv, dgate, (hipStream_t)stream);
}

int edet_se_fwd(int B, int C, int R, const float* s, const float* w1, const float* b1,
                const float* w2, const float* b2, float* z1, float* gate, edet_stream_t stream) {
  EDET_REQUIRE(s && w1 && b1 && w2 && b2 && z1 && gate && B > 0 && C > 0 && R > 0,
               "se_fwd: bad argument");
  hipLaunchKernelGGL(k_se_fwd, dim3(B), dim3(256), (C + R) * sizeof(float), (hipStream_t)stream, C, R, s,
                     w1, b1, w2, b2, z1, gate);
  return check_launch("edet se_fwd");
}

int edet_se_bwd(int B, int C, int R, int HW, const float* s, const float* z1,
                const float* gate, const float* dgate, const float* w1, const float* w2,
                float* dw1, float* db1, float* dw2, float* db2, float* dsq,
                edet_stream_t stream) {
  EDET_REQUIRE(s && z1 && gate && dgate && w1 && w2 && dw1 && db1 && dw2 && db2 && dsq,
               "se_bwd: null argument");
  hipLaunchKernelGGL(k_se_bwd, dim3(B), dim3(256), (2 * C + 2 * R) * sizeof(float), (hipStream_t)stream,
                     C, R, HW, s, z1, gate, dgate, w1, w2, dw1, db1, dw2, db2, dsq);
  return check_launch("edet se_bwd");
}

int edet_residual_fwd(int dtype, const edet_lazy* x, const edet_lazy* res,
                      const edet_pyramid* p, int C, const float* scale, void* out,
                      edet_stream_t stream) {
  int rc = lazy_checks(x, p, C);
  if (rc) return rc;
  rc = lazy_checks(res, p, C);
  if (rc) return rc;
  EDET_REQUIRE(out, "residual_fwd: null out");
  LArgs g{};
  g.lz = *x; g.res = *res; g.p = *p; g.dv_scale = scale; g.dx = out; g.C = C;
  g.ncb = cdiv(C, RCB);
  const int nb = total_chunks(*p, RCH) * g.ncb;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) hipLaunchKernelGGL(k_residual<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, g);
    return check_launch("edet residual");
  });
}

int edet_bn_inference_stats(int64_t n, const float* mmean, const float* mvar, const float* count,
                            float* sum, float* sq, edet_stream_t stream) {
  EDET_REQUIRE(mmean && mvar && count && sum && sq, "bn_inference_stats: null argument");
  if (n <= 0) return EDET_OK;
  hipLaunchKernelGGL(k_bn_infer_stats, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     mmean, mvar, count, sum, sq);
  return check_launch("edet bn_inference_stats");
}

int edet_bn_update_moving(int64_t n, const float* sum, const float* sq, const float* count,
                          float momentum, float* mmean, float* mvar, edet_stream_t stream) {
  EDET_REQUIRE(sum && sq && count && mmean && mvar, "bn_update_moving: null argument");
  if (n <= 0) return EDET_OK;
  hipLaunchKernelGGL(k_bn_update, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     n, sum, sq, count, momentum, mmean, mvar);
  return check_launch("edet bn_update_moving");
}

}  // extern "C"
