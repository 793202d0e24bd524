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

// Row kernels: a block covers R full rows per pass with TPR threads per row (TPR = C/8
// 8-channel vectors, or 256 for C > 2048 with up to 2 vectors per thread), so every pass is
// R contiguous rows of the NHWC tensor (fully coalesced, no idle lanes for C = 96/144/240...)
// and each thread keeps a fixed channel vector -> per-thread partial sums need no atomics.
constexpr int RVPT = 2;  // vectors per thread (C <= 4096)
// rows per trip in the streaming row loops: both rows' loads are issued before either is
// consumed (in apply, before either store: vmcnt orders loads behind earlier stores)
constexpr int EU = 2;
// the reduce-type row kernels (BN-backward reduce, SE squeeze, SE-fused BN reduce) and the
// materialize pass take four rows per trip (reduce 1.59 -> 1.51, materialize 0.61 -> 0.58
// ms/step); apply is unchanged at four.  The SE-fused reduce was slower at four with ~8-pass
// chunks and is faster (561 -> 542 us) at its 16-pass chunks.
constexpr int EUR = 4;

struct RowGeom {
  int TPR, R, VPT, CH;  // threads per row, rows per pass, vectors per thread, rows per chunk
};

// passes: rows per chunk = R * passes; 0 = about 16K elements per chunk (at most 16 passes)
static RowGeom row_geom(int C, int passes = 0) {
  RowGeom r;
  const int NV = C / 8;
  r.TPR = NV <= 256 ? NV : 256;
  r.VPT = cdiv(NV, r.TPR);
  r.R = 256 / r.TPR;
  if (passes <= 0) {
    passes = 16384 / (r.R * C);
    // C >= 1024 runs one row per block pass: shorter chunks give more blocks in flight
    // (M = 8192, C = 1152 apply: 38 -> 31 us, scripts/row_probe.py)
    if (C >= 1024 && passes > 8) passes = 8;
  }
  if (passes < 1) passes = 1;
  if (passes > 32) passes = 32;
  r.CH = r.R * passes;
  return r;
}

struct LArgs {
  edet_lazy lz;
  edet_lazy res;
  edet_pyramid p;
  edet_bngrad64 acc;   // fp64 dgamma / dbeta accumulators (reduce -> apply)
  edet_segout grads;   // fp32 parameter gradients (apply, block of chunk 0 per segment)
  int has_grads;
  const void* dv;
  void* dx;
  const float* dv_scale;
  const float* dsq;
  double* out64;  // se_squeeze / gate_grad output [batch][C]
  int C, accumulate, hw, chunks_per_img;
  RowGeom geo;
  int cslices;  // k_gate_bn_reduce: channel slices of geo.TPR * 8 channels (1 = whole rows)
};

// per-channel tables in dynamic LDS: af (sc, sh), mr (mean, rstd), gb (dgamma/M, dbeta/M), for
// channels [c_lo, c_hi) (a block's channel slice) at their channel index.  One channel per
// thread and trip, its replicas' loads (common.hpp stat_idx: 4 statistics vectors x 4
// replicas) all issued before any is used -- 32 VGPRs in flight; the two-channel form of round
// 5 held twice that once the statistics were replicated and cost the apply kernels 1-3 waves
// per SIMD (r06k: 80-114 -> 138 VGPRs).
__device__ __forceinline__ void load_tables(const edet_lazy& lz, int seg, float inv, int c_lo, int c_hi, float2* af,
                                            float2* mr, float2* gb, const edet_bngrad64* acc) {
  const bool bn = lz.bn.enabled;
  for (int c = c_lo + threadIdx.x; c < c_hi; c += blockDim.x) {
    float2 a = make_float2(1.f, 0.f), b = make_float2(0.f, 1.f), d = make_float2(0.f, 0.f);
    if (bn) {  // bn_affine / bn_mean_rstd (common.hpp), the same arithmetic
      double su[SR], sq[SR], dg[SR], db[SR];
      const int i = stat_idx(c, 0);
#pragma unroll
      for (int r = 0; r < SR; ++r) {
        su[r] = lz.bn.sum[seg][i + 16 * r];
        sq[r] = lz.bn.sq[seg][i + 16 * r];
        if (gb) {
          dg[r] = acc->dgamma[seg][i + 16 * r];
          db[r] = acc->dbeta[seg][i + 16 * r];
        }
      }
      const float ga = lz.bn.gamma[seg][c], be = lz.bn.beta[seg][c];
      const double mean = ((su[0] + su[1]) + (su[2] + su[3])) * (double)inv;
      const double var = fmax(((sq[0] + sq[1]) + (sq[2] + sq[3])) * (double)inv - mean * mean, 0.0);
      const float r = rsqrtf((float)var + lz.bn.eps);
      const float sc = ga * r;
      a = make_float2(sc, be - (float)mean * sc);
      b = make_float2((float)mean, r);
      if (gb)
        d = make_float2((float)(((dg[0] + dg[1]) + (dg[2] + dg[3])) * (double)inv),
                        (float)(((db[0] + db[1]) + (db[2] + db[3])) * (double)inv));
    }
    af[c] = a;
    if (mr) mr[c] = b;
    if (gb) gb[c] = d;
  }
}

// Persistent over chunks (block b takes chunks b, b+grid, ...): per-thread partials live in
// registers until the segment changes, so each block issues 2C atomics per segment.
template <typename T>
__device__ __forceinline__ void flush_reduce(const LArgs& g, const RowGeom& geo, int seg, int rr, int tv, float* red,
                                             float (&s)[RVPT][8], float (&q)[RVPT][8]) {
  const int C = g.C, NV = C / 8, tid = threadIdx.x;
  if (rr < geo.R) {
#pragma unroll
    for (int v = 0; v < RVPT; ++v) {
      const int cv = tv + v * geo.TPR;
      if (v < geo.VPT && cv < NV) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red[(0 * geo.R + rr) * C + cv * 8 + j] = s[v][j];
          red[(1 * geo.R + rr) * C + cv * 8 + j] = q[v][j];
        }
      }
    }
  }
#pragma unroll
  for (int v = 0; v < RVPT; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[v][j] = 0.f; q[v][j] = 0.f; }
  __syncthreads();
  for (int c = tid; c < C; c += blockDim.x) {
    float ss = 0.f, qq = 0.f;
    for (int i = 0; i < geo.R; ++i) { ss += red[i * C + c]; qq += red[(geo.R + i) * C + c]; }
    stat_put(g.acc.dbeta[seg], c, (double)ss);
    stat_put(g.acc.dgamma[seg], c, (double)qq);
  }
  __syncthreads();
}

// compile-time cases of the lazy backward row kernels
// AF_DVS: a per-image drop-connect scale of dv; AF_ACC (apply): dx accumulates.  Compile-time,
// so the row loop has no load under a runtime branch (the compiler's wait counts then drained
// every row's loads: s_waitcnt vmcnt(0) in the loop)
enum { AF_BN = 1, AF_ACT = 2, AF_GATE = 4, AF_DSQ = 8, AF_DVS = 16, AF_ACC = 32 };

// streaming (nontemporal) 16-byte row accesses for the applies over tensors far larger than the
// caches (development slot 53 = 1)
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld8_nt(const uint16_t* p, float* o) {
  const u32x4_nt v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8_nt(uint16_t* p, const float* v) {
  u32x4_nt w;
  w.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  w.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  w.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
  w.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
  __builtin_nontemporal_store(w, reinterpret_cast<u32x4_nt*>(p));
}

template <typename T, int F>
__global__ __launch_bounds__(256) void k_lazy_bwd_reduce(LArgs g, int nchunks) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = g.C;
  float2* af = reinterpret_cast<float2*>(smem);
  float2* mr = af + C;
  float* red = reinterpret_cast<float*>(mr + C);  // [2][R][C]
  const RowGeom geo = g.geo;
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  const int NV = C / 8;
  float s[RVPT][8], q[RVPT][8];
#pragma unroll
  for (int v = 0; v < RVPT; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[v][j] = 0.f; q[v][j] = 0.f; }
  int cur_seg = -1;
  for (int b = blockIdx.x; b < nchunks; b += gridDim.x) {
    int seg, chunk;
    chunk_lookup(g.p, geo.CH, b, seg, chunk);
    const int rows = seg_rows(g.p, seg);
    if (seg != cur_seg) {
      if (cur_seg >= 0) flush_reduce<T>(g, geo, cur_seg, rr, tv, red, s, q);
      load_tables(g.lz, seg, 1.f / (float)rows, 0, C, af, mr, nullptr, nullptr);
      cur_seg = seg;
      __syncthreads();
    }
    const int off = g.p.row_off[seg];
    const int m_begin = off + chunk * geo.CH, m_end = min(off + rows, m_begin + geo.CH);
    const int hw = g.p.H[seg] * g.p.W[seg];
    const float* dvsp = g.dv_scale ? g.dv_scale + seg * g.p.batch : nullptr;
    if (rr < geo.R) {
#pragma unroll
      for (int v = 0; v < RVPT; ++v) {
        const int cv = tv + v * geo.TPR;
        if (!(v < geo.VPT && cv < NV)) continue;
        const int c = cv * 8;
        // the 8 channels' tables in registers for the whole chunk (as k_lazy_bwd_apply)
        float sc[8], sh[8], mu_[8], rs[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float2 a = af[c + j], r = mr[c + j];
          sc[j] = a.x; sh[j] = a.y; mu_[j] = r.x; rs[j] = r.y;
        }
        for (int m = m_begin + rr; m < m_end; m += EUR * geo.R) {
          float x[EUR][8], d[EUR][8], gt[EUR][8], ds[EUR][8], dvs[EUR];
#pragma unroll
          for (int u = 0; u < EUR; ++u) {
            const int mu = min(m + u * geo.R, m_end - 1);
            const int n = (mu - off) / hw;
            ld8((const T*)g.lz.x + (size_t)mu * g.lz.ld + c, x[u]);
            ld8((const T*)g.dv + (size_t)mu * C + c, d[u]);
            dvs[u] = (F & AF_DVS) ? dvsp[n] : 1.f;
            if (F & AF_GATE) ld8(g.lz.gate + (size_t)n * C + c, gt[u]);
            if (F & AF_DSQ) ld8(g.dsq + (size_t)n * C + c, ds[u]);
          }
#pragma unroll
          for (int u = 0; u < EUR; ++u) {
            const float k = m + u * geo.R < m_end ? dvs[u] : 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float gg = d[u][j] * k;
              if (F & AF_GATE) gg *= gt[u][j];
              if (F & AF_DSQ) gg += ds[u][j] * (k != 0.f ? 1.f : 0.f);
              const float du = (F & AF_ACT) ? gg * dswishf_(x[u][j] * sc[j] + sh[j]) : gg;
              s[v][j] += du;
              q[v][j] += du * ((x[u][j] - mu_[j]) * rs[j]);
            }
          }
        }
      }
    }
  }
  if (cur_seg >= 0) flush_reduce<T>(g, geo, cur_seg, rr, tv, red, s, q);
}

// Persistent over chunks like the reduce (block b takes chunks b, b+grid, ...): the
// per-channel tables (fp64 statistics -> affine, mean/rstd, dgamma/M, dbeta/M) are rebuilt
// only when the segment changes.  The BN / swish / gate / dsq cases are compile-time (F) and
// each thread folds its 8 channels' tables into registers once per chunk:
//   u = x*sc + sh,   dx = sc*du + kb*x + kc   with kb = -sc*rstd*dgamma/M,
//   kc = -sc*dbeta/M + sc*rstd*mean*dgamma/M   (= sc*(du - dbeta/M - xhat*dgamma/M))
// so the row loop is loads, ~10 VALU per element and stores (no LDS, no per-element branches).
template <typename T, int F, bool NT = false>
__global__ __launch_bounds__(256) void k_lazy_bwd_apply(LArgs g, int nchunks) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = g.C;
  float2* af = reinterpret_cast<float2*>(smem);
  float2* mr = af + C;
  float2* gb = mr + C;
  const RowGeom geo = g.geo;
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  const int NV = C / 8;
  T* DX = (T*)g.dx;
  // channel slices (g.cslices > 1, the wide short tensors): work item b = (chunk, slice); a
  // block builds the tables of its slice only (all C of them per 8-row chunk cost more than the
  // chunk's rows once the statistics were replicated)
  const int ns = g.cslices, CSW = ns > 1 ? geo.TPR * 8 : C;
  int cur_seg = -1, cur_cs = -1;
  for (int b = blockIdx.x; b < nchunks * ns; b += gridDim.x) {
    const int cs = b % ns;
    int seg, chunk;
    chunk_lookup(g.p, geo.CH, b / ns, seg, chunk);
    const int rows = seg_rows(g.p, seg);
    const int c_lo = cs * CSW, c_hi = min(C, c_lo + CSW);
    if (seg != cur_seg || cs != cur_cs) {
      if (cur_seg >= 0) __syncthreads();  // the previous tables are still being read
      load_tables(g.lz, seg, 1.f / (float)rows, c_lo, c_hi, af, mr, gb, &g.acc);
      cur_seg = seg;
      cur_cs = cs;
      __syncthreads();
    }
    if (g.has_grads && chunk == 0)  // one writer per segment and channel: fp32 parameter gradients
      for (int c = c_lo + threadIdx.x; c < c_hi; c += blockDim.x) {
        g.grads.a[seg][c] += (float)stat_get(g.acc.dgamma[seg], c);
        g.grads.b[seg][c] += (float)stat_get(g.acc.dbeta[seg], c);
      }
    if (rr >= geo.R) continue;
    const int off = g.p.row_off[seg];
    const int m_begin = off + chunk * geo.CH, m_end = min(off + rows, m_begin + geo.CH);
    const int hw = g.p.H[seg] * g.p.W[seg];
    const float* dvsp = g.dv_scale ? g.dv_scale + seg * g.p.batch : nullptr;
#pragma unroll
    for (int v = 0; v < RVPT; ++v) {
      const int cv = c_lo / 8 + tv + v * geo.TPR;
      if (!(v < geo.VPT && cv < NV)) continue;
      const int c = cv * 8;
      float sc[8], sh[8], kb[8], kc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float2 a = af[c + j];
        sc[j] = a.x; sh[j] = a.y;
        if (F & AF_BN) {
          const float2 q = mr[c + j], d = gb[c + j];
          kb[j] = -a.x * q.y * d.x;
          kc[j] = -a.x * d.y - kb[j] * q.x;
        }
      }
      // EU rows per trip, all loads before any store (vmcnt orders loads behind earlier stores)
      for (int m = m_begin + rr; m < m_end; m += EU * geo.R) {
        float x[EU][8], d[EU][8], gt[EU][8], ds[EU][8], dvs[EU];
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          const int mu = min(m + u * geo.R, m_end - 1);
          const int n = (mu - off) / hw;
          if constexpr (NT && sizeof(T) == 2) {
            ld8_nt((const uint16_t*)g.lz.x + (size_t)mu * g.lz.ld + c, x[u]);
            ld8_nt((const uint16_t*)g.dv + (size_t)mu * C + c, d[u]);
          } else {
            ld8((const T*)g.lz.x + (size_t)mu * g.lz.ld + c, x[u]);
            ld8((const T*)g.dv + (size_t)mu * C + c, d[u]);
          }
          dvs[u] = (F & AF_DVS) ? dvsp[n] : 1.f;
          if (F & AF_GATE) ld8(g.lz.gate + (size_t)n * C + c, gt[u]);
          if (F & AF_DSQ) ld8(g.dsq + (size_t)n * C + c, ds[u]);
        }
#pragma unroll
        for (int u = 0; u < EU; ++u) {
          const int mu = m + u * geo.R;
          if (mu >= m_end) break;
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float gg = d[u][j] * dvs[u];
            if (F & AF_GATE) gg *= gt[u][j];
            if (F & AF_DSQ) gg += ds[u][j];
            const float du = (F & AF_ACT) ? gg * dswishf_(x[u][j] * sc[j] + sh[j]) : gg;
            o[j] = (F & AF_BN) ? sc[j] * du + kb[j] * x[u][j] + kc[j] : du;
          }
          if constexpr (NT && sizeof(T) == 2 && !(F & AF_ACC)) st8_nt((uint16_t*)(DX + (size_t)mu * C + c), o);
          else acc8m(DX + (size_t)mu * C + c, 8, o, (F & AF_ACC) ? 1 : 0);
        }
      }
    }
  }
}

// out[n][c] += (scale) * sum_hw f(row)   -- SE squeeze (mean of v(x)) or gate grad (dv * v(x))
template <typename T, bool GATEGRAD, bool ACT>
__global__ __launch_bounds__(256) void k_img_reduce(LArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = g.C;
  float2* af = reinterpret_cast<float2*>(smem);
  const RowGeom geo = g.geo;
  // channel slices (as k_gate_bn_reduce): block = (image, slice of geo.TPR vectors), VPT = 1
  const int CSW = g.cslices > 1 ? geo.TPR * 8 : C;
  float* red = reinterpret_cast<float*>(af + C);  // [R][CSW]
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  const int cs = blockIdx.x % g.cslices, bi = blockIdx.x / g.cslices;
  const int n = bi / g.chunks_per_img, chunk = bi - n * g.chunks_per_img;
  const int cvb = cs * geo.TPR;
  load_tables(g.lz, 0, 1.f / (float)seg_rows(g.p, 0), cvb * 8, min(C, cvb * 8 + CSW), af, nullptr, nullptr, nullptr);
  __syncthreads();
  const int m_begin = n * g.hw + chunk * geo.CH, m_end = min((n + 1) * g.hw, m_begin + geo.CH);
  const int NV = C / 8;
  float s[RVPT][8];
#pragma unroll
  for (int v = 0; v < RVPT; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[v][j] = 0.f;
  if (rr < geo.R) {
#pragma unroll
    for (int v = 0; v < RVPT; ++v) {
      const int cv = cvb + tv + v * geo.TPR;
      if (!(v < geo.VPT && cv < NV)) continue;
      const int c = cv * 8;
      float2 a8[8];  // the 8 channels' affine in registers
#pragma unroll
      for (int j = 0; j < 8; ++j) a8[j] = af[c + j];
      for (int m = m_begin + rr; m < m_end; m += EUR * geo.R) {
        float x[EUR][8], d[EUR][8];
#pragma unroll
        for (int u = 0; u < EUR; ++u) {
          const int mu = min(m + u * geo.R, m_end - 1);
          ld8((const T*)g.lz.x + (size_t)mu * g.lz.ld + c, x[u]);
          if (GATEGRAD) ld8((const T*)g.dv + (size_t)mu * C + c, d[u]);
        }
#pragma unroll
        for (int u = 0; u < EUR; ++u) {
          const float k = m + u * geo.R < m_end ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float val = lazy_apply(x[u][j], a8[j], ACT) * k;
            s[v][j] += GATEGRAD ? d[u][j] * val : val;
          }
        }
      }
    }
#pragma unroll
    for (int v = 0; v < RVPT; ++v) {
      const int cv = cvb + tv + v * geo.TPR;
      if (v < geo.VPT && cv < NV)
#pragma unroll
        for (int j = 0; j < 8; ++j) red[rr * CSW + (cv - cvb) * 8 + j] = s[v][j];
    }
  }
  __syncthreads();
  // a block over the whole image owns its (image, channel) outputs: read-add-write, no atomics
  const bool owner = g.chunks_per_img == 1;
  for (int cc = tid; cc < CSW; cc += blockDim.x) {
    const int c = cvb * 8 + cc;
    if (c >= C) break;
    float ss = 0.f;
    for (int i = 0; i < geo.R; ++i) ss += red[i * CSW + cc];
    const double val = GATEGRAD ? (double)ss : (double)ss / (double)g.hw;
    double* o = g.out64 + (size_t)n * C + c;
    if (owner) *o += val;
    else atomicAdd(o, val);
  }
}

// SE-gated value v = swish(u) * gate, u = bn(x): one pass over (x, dv) yields, per image and
// channel, everything the SE backward and the BN backward reduction need:
//   [0] sum dv*swish(u)             -> d gate (the gate gradient, as k_img_reduce<T, true>)
//   [1] sum dv*swish'(u)  [2] sum swish'(u)  [3] sum dv*swish'(u)*xhat  [4] sum swish'(u)*xhat
// Since du = (dv*gate + dsq) * swish'(u) with gate and dsq constant per (image, channel),
//   dbeta = sum_n gate*[1] + dsq*[2],  dgamma = sum_n gate*[3] + dsq*[4]   (k_se_bn_combine)
// which replaces the separate k_lazy_bwd_reduce pass over x and dv for these tensors.
template <typename T>
__global__ __launch_bounds__(256) void k_gate_bn_reduce(LArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = g.C;
  float2* af = reinterpret_cast<float2*>(smem);
  float2* mr = af + C;
  const RowGeom geo = g.geo;
  const int CSW = geo.TPR * 8;  // channels of this block's slice (all of C when cslices == 1)
  float* red = reinterpret_cast<float*>(mr + C);  // [R][CSW] per quantity, reused 5 times
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  const int cs = blockIdx.x % g.cslices, bi = blockIdx.x / g.cslices;
  const int n = bi / g.chunks_per_img, chunk = bi - n * g.chunks_per_img;
  load_tables(g.lz, 0, 1.f / (float)seg_rows(g.p, 0), cs * CSW, min(C, cs * CSW + CSW), af, mr, nullptr, nullptr);
  __syncthreads();
  const int m_begin = n * g.hw + chunk * geo.CH, m_end = min((n + 1) * g.hw, m_begin + geo.CH);
  const int c0 = cs * CSW, c = c0 + tv * 8;
  const bool live = rr < geo.R && c < C;
  float a[5][8];
#pragma unroll
  for (int q = 0; q < 5; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[q][j] = 0.f;
  if (live) {
    float sc[8], sh[8], mu_[8], rs[8];  // the 8 channels' tables in registers
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float2 t = af[c + j], b = mr[c + j];
      sc[j] = t.x; sh[j] = t.y; mu_[j] = b.x; rs[j] = b.y;
    }
    for (int m = m_begin + rr; m < m_end; m += EUR * geo.R) {
      float x[EUR][8], d[EUR][8];
#pragma unroll
      for (int u = 0; u < EUR; ++u) {
        const int mu = min(m + u * geo.R, m_end - 1);
        ld8((const T*)g.lz.x + (size_t)mu * g.lz.ld + c, x[u]);
        ld8((const T*)g.dv + (size_t)mu * C + c, d[u]);
      }
#pragma unroll
      for (int u = 0; u < EUR; ++u) {
        const float k = m + u * geo.R < m_end ? 1.f : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float uu = x[u][j] * sc[j] + sh[j];
          const float sg = sigmoidf_(uu);
          const float sw = uu * sg, dsw = sg * (1.f + uu * (1.f - sg)) * k;
          const float xh = (x[u][j] - mu_[j]) * rs[j];
          const float dd = d[u][j] * k;
          a[0][j] += dd * sw;
          a[1][j] += dd * dsw;
          a[2][j] += dsw;
          a[3][j] += dd * dsw * xh;
          a[4][j] += dsw * xh;
        }
      }
    }
  }
  // one block per (image, slice) over the whole image owns its outputs: plain read-add-write
  // instead of fp64 atomics (C = 1152: 5C atomics from each of 8 blocks per image)
  const bool owner = g.chunks_per_img == 1;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    __syncthreads();
    if (live)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[rr * CSW + tv * 8 + j] = a[q][j];
    __syncthreads();
    for (int cc = tid; cc < CSW; cc += blockDim.x) {
      if (c0 + cc >= C) break;
      float ss = 0.f;
      for (int i = 0; i < geo.R; ++i) ss += red[i * CSW + cc];
      double* o = g.out64 + ((size_t)q * g.p.batch + n) * C + c0 + cc;
      if (owner) *o += (double)ss;
      else atomicAdd(o, (double)ss);
    }
  }
}

// a half-wave per channel, its lanes over the images (one thread looping B images was B
// dependent load rounds on a handful of blocks); `blk` = this block's index among the combine's
template <bool DSQ_FROM_DZ1>
__device__ __forceinline__ void se_bn_combine_body(int B, int C, int blk, const float* gate, const float* dsq,
                                                   const double* s5, double* dgamma, double* dbeta, int R = 0,
                                                   int HW = 1, const float* dz1 = nullptr,
                                                   const float* w1 = nullptr) {
  const int half = threadIdx.x >> 5, ln = threadIdx.x & 31;
  const int c = blk * 8 + half;
  double gb = 0.0, gg = 0.0;
  if (c < C)
    for (int n = ln; n < B; n += 32) {
      double ds;
      if constexpr (DSQ_FROM_DZ1) {  // k_se_wgrad's dsq loop, same order
        float a = 0.f;
#pragma unroll 8
        for (int r = 0; r < R; ++r) a += dz1[(size_t)n * R + r] * w1[(size_t)r * C + c];
        ds = a / (float)HW;
      } else {
        ds = dsq[(size_t)n * C + c];
      }
      const double gt = gate[(size_t)n * C + c];
      const size_t i = (size_t)n * C + c, BC = (size_t)B * C;
      gb += gt * s5[1 * BC + i] + ds * s5[2 * BC + i];
      gg += gt * s5[3 * BC + i] + ds * s5[4 * BC + i];
    }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    gb += __shfl_xor(gb, o, 64);
    gg += __shfl_xor(gg, o, 64);
  }
  if (c < C && ln == 0) {  // the channel's one writer: replica 0
    dbeta[stat_idx(c, 0)] += gb;
    dgamma[stat_idx(c, 0)] += gg;
  }
}

__global__ __launch_bounds__(256) void k_se_bn_combine(int B, int C, const float* gate, const float* dsq,
                                                       const double* s5, double* dgamma, double* dbeta) {
  se_bn_combine_body<false>(B, C, (int)blockIdx.x, gate, dsq, s5, dgamma, dbeta);
}

// SE excite: z1 = W1 s + b1 ; gate = sigmoid(W2 swish(z1) + b2)   (layers/se.py:36-39).
// The excite is tiny (B x C x R MACs) but was one block per image; it is now spread over the
// chip: one wave per (n, r) dot product over C, then one thread per (n, c) over R.  Every
// output (including the weight gradients) has exactly one writer: no atomics, reproducible.

// z1[n][r] = sum_c w1[r][c] s[n][c] + b1[r]     (one wave per (n, r))
__global__ __launch_bounds__(256) void k_se_reduce_c(int B, int C, int R, const double* s, const float* w1,
                                                     const float* b1, float* z1) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= B * R) return;
  const int n = item / R, r = item - n * R;
  float a = 0.f;
#pragma unroll 4
  for (int c = lane; c < C; c += 64) a += w1[(size_t)r * C + c] * (float)s[(size_t)n * C + c];
  a = wave_sum(a);
  if (lane == 0) z1[item] = a + b1[r];
}

// gate[n][c] = sigmoid(sum_r w2[c][r] swish(z1[n][r]) + b2[c])   (one thread per (n, c))
__global__ __launch_bounds__(256) void k_se_excite(int B, int C, int R, const float* z1, const float* w2,
                                                   const float* b2, float* gate) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= B * C) return;
  const int n = idx / C, c = idx - n * C;
  float a = b2[c];
#pragma unroll 8
  for (int r = 0; r < R; ++r) {
    const float z = z1[(size_t)n * R + r];
    a += w2[(size_t)c * R + r] * (z * sigmoidf_(z));
  }
  gate[idx] = sigmoidf_(a);
}

// backward, pass 1: dz1[n][r] = swish'(z1) * sum_c dz2[n][c] w2[c][r],
// dz2 = dgate * g (1 - g)   (one wave per (n, r))
__global__ __launch_bounds__(256) void k_se_dz1(int B, int C, int R, const float* z1, const float* gate,
                                                const double* dgate, const float* w2, float* dz1) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= B * R) return;
  const int n = item / R, r = item - n * R;
  float a = 0.f;
#pragma unroll 4
  for (int c = lane; c < C; c += 64) {
    const float gv = gate[(size_t)n * C + c];
    a += (float)dgate[(size_t)n * C + c] * gv * (1.f - gv) * w2[(size_t)c * R + r];
  }
  a = wave_sum(a);
  if (lane == 0) {
    const float z = z1[item];
    const float sg = sigmoidf_(z);
    dz1[item] = a * sg * (1.f + z * (1.f - sg));
  }
}

// backward, pass 2 (dw2 / dw1: a block per 32 channels, the images staged in LDS; dsq, db2,
// db1: a thread per element):
//   dw2[c][r] += sum_n dz2[n][c] swish(z1[n][r])     dw1[r][c] += sum_n dz1[n][r] s[n][c]
//   db2[c]    += sum_n dz2[n][c]                     db1[r]    += sum_n dz1[n][r]
//   dsq[n][c]  = sum_r dz1[n][r] w1[r][c] / HW
// The weight gradients are (C x B)(B x R) products: a block per 32 channels x 8 r stages dz2
// and s of its channels and swish(z1), dz1 of its r, 32 images at a time (coalesced rows), and
// thread (c, r) accumulates both products over the images (the former half-wave per (c, r) read
// gate / dgate / s with stride C across its lanes: 12 us per launch at C = 1152, R = 48).
constexpr int SEW_NB = 32, SEW_C = 32, SEW_R = 8;
__host__ __device__ inline int se_wgrad_blocks(int C, int R) { return cdiv(C, SEW_C) * cdiv(R, SEW_R); }
__device__ __forceinline__ void k_se_wgrad_body(int B, int C, int R, int HW, int nA, const double* s,
                                                const float* z1, const float* gate, const double* dgate,
                                                const float* dz1, const float* w1, float* dw1, float* db1,
                                                float* dw2, float* db2, float* dsq) {
  if ((int)blockIdx.x < nA) {
    __shared__ float d2s[SEW_NB][SEW_C], svs[SEW_NB][SEW_C], zss[SEW_NB][SEW_R], dzs[SEW_NB][SEW_R];
    const int tid = threadIdx.x, cl = tid & 31, rl = tid >> 5;
    const int nrt = cdiv(R, SEW_R);
    const int c0 = ((int)blockIdx.x / nrt) * SEW_C, r0 = ((int)blockIdx.x % nrt) * SEW_R;
    const int c = c0 + cl, r = r0 + rl;
    float a2 = 0.f, a1 = 0.f;
    for (int n0 = 0; n0 < B; n0 += SEW_NB) {
      const int nb = min(SEW_NB, B - n0);
      __syncthreads();
#pragma unroll
      for (int u = 0; u < SEW_NB * SEW_C / 256; ++u) {  // clamped addresses, values selected
        const int e = tid + u * 256, n = e >> 5, cc = c0 + (e & 31);
        const bool ok = n < nb && cc < C;
        const size_t i = ok ? (size_t)(n0 + n) * C + cc : 0;
        const float gv = gate[i];
        const double dg = dgate[i], sv = s[i];
        d2s[n][e & 31] = ok ? (float)dg * gv * (1.f - gv) : 0.f;
        svs[n][e & 31] = ok ? (float)sv : 0.f;
      }
      {
        const int n = tid >> 3, rr = r0 + (tid & 7);
        const bool ok = n < nb && rr < R;
        const size_t i = ok ? (size_t)(n0 + n) * R + rr : 0;
        const float z = z1[i], d = dz1[i];
        zss[n][tid & 7] = ok ? z * sigmoidf_(z) : 0.f;
        dzs[n][tid & 7] = ok ? d : 0.f;
      }
      __syncthreads();
#pragma unroll 8
      for (int n = 0; n < nb; ++n) {
        a2 += d2s[n][cl] * zss[n][rl];
        a1 += dzs[n][rl] * svs[n][cl];
      }
    }
    if (r < R && c < C) {
      dw2[(size_t)c * R + r] += a2;
      dw1[(size_t)r * C + c] += a1;
    }
    return;
  }
  const int idx = (blockIdx.x - nA) * 256 + threadIdx.x;
  if (idx < B * C) {
    const int n = idx / C, c = idx - n * C;
    float a = 0.f;
#pragma unroll 8
    for (int r = 0; r < R; ++r) a += dz1[(size_t)n * R + r] * w1[(size_t)r * C + c];
    dsq[idx] = a / (float)HW;
  }
  if (idx < C) {
    float a = 0.f;
#pragma unroll 8
    for (int n = 0; n < B; ++n) {
      const float gv = gate[(size_t)n * C + idx];
      a += (float)dgate[(size_t)n * C + idx] * gv * (1.f - gv);
    }
    db2[idx] += a;
  }
  if (idx < R) {
    float a = 0.f;
#pragma unroll 8
    for (int n = 0; n < B; ++n) a += dz1[(size_t)n * R + idx];
    db1[idx] += a;
  }
}

__global__ __launch_bounds__(256) void k_se_wgrad(int B, int C, int R, int HW, int nA, const double* s,
                                                  const float* z1, const float* gate, const double* dgate,
                                                  const float* dz1, const float* w1, float* dw1, float* db1,
                                                  float* dw2, float* db2, float* dsq) {
  k_se_wgrad_body(B, C, R, HW, nA, s, z1, gate, dgate, dz1, w1, dw1, db1, dw2, db2, dsq);
}

// k_se_wgrad with k_se_bn_combine's blocks appended (nW = k_se_wgrad's grid).  dsq is written
// by the k_se_wgrad blocks of the same launch, so the combine blocks re-derive the dsq values
// they need from dz1 (final after k_se_dz1) with the same loop, bit for bit, instead of
// taking a launch of their own
__global__ __launch_bounds__(256) void k_se_wgrad_bn(int B, int C, int R, int HW, int nA, int nW, const double* s,
                                                     const float* z1, const float* gate, const double* dgate,
                                                     const float* dz1, const float* w1, float* dw1, float* db1,
                                                     float* dw2, float* db2, float* dsq, const double* s5,
                                                     double* dgamma, double* dbeta) {
  if ((int)blockIdx.x < nW) {
    k_se_wgrad_body(B, C, R, HW, nA, s, z1, gate, dgate, dz1, w1, dw1, db1, dw2, db2, dsq);
    return;
  }
  se_bn_combine_body<true>(B, C, (int)blockIdx.x - nW, gate, dsq, s5, dgamma, dbeta, R, HW, dz1, w1);
}

// heads: out = v(x) * scale[seg][n] + v(res)   (class_net.py:93-96 with drop_connect.py:4-18)
template <typename T>
__global__ __launch_bounds__(256) void k_residual(LArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = g.C;
  float2* ax = reinterpret_cast<float2*>(smem);
  float2* ar = ax + C;
  const RowGeom geo = g.geo;
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  int seg, chunk;
  chunk_lookup(g.p, geo.CH, blockIdx.x, seg, chunk);
  const int rows = seg_rows(g.p, seg);
  const float inv = 1.f / (float)rows;
  load_tables(g.lz, seg, inv, 0, C, ax, nullptr, nullptr, nullptr);
  load_tables(g.res, seg, inv, 0, C, ar, nullptr, nullptr, nullptr);
  __syncthreads();
  if (rr >= geo.R) return;
  const int off = g.p.row_off[seg];
  const int m_begin = off + chunk * geo.CH, m_end = min(off + rows, m_begin + geo.CH);
  const int hw = g.p.H[seg] * g.p.W[seg];
  const int NV = C / 8;
  T* OUT = (T*)g.dx;
  for (int m = m_begin + rr; m < m_end; m += geo.R) {
    const int n = (m - off) / hw;
    const float sc = g.dv_scale ? g.dv_scale[seg * g.p.batch + n] : 1.f;
#pragma unroll
    for (int v = 0; v < RVPT; ++v) {
      const int cv = tv + v * geo.TPR;
      if (v < geo.VPT && cv < NV) {
        const int c = cv * 8;
        float x[8], r[8], o[8];
        ld8((const T*)g.lz.x + (size_t)m * g.lz.ld + c, x);
        ld8((const T*)g.res.x + (size_t)m * g.res.ld + c, r);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          o[j] = lazy_apply(x[j], ax[c + j], g.lz.act) * sc + lazy_apply(r[j], ar[c + j], g.res.act);
        st8(OUT + (size_t)m * C + c, o);
      }
    }
  }
}

// out = v(x) = act(bn(x)) * gate, written once.  Used for the SE-gated depthwise output that
// both the project conv's forward GEMM and its weight gradient read: applying the transform in
// their A-operand loads cost more than this extra pass (it was recomputed per column tile).
template <typename T, bool ACT, bool GATE>
__global__ __launch_bounds__(256) void k_materialize(LArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int C = g.C;
  float2* ax = reinterpret_cast<float2*>(smem);
  const RowGeom geo = g.geo;
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  // channel slices (as the apply): block = (chunk, slice), tables of the slice only
  const int ns = g.cslices, CSW = ns > 1 ? geo.TPR * 8 : C, cs = blockIdx.x % ns;
  int seg, chunk;
  chunk_lookup(g.p, geo.CH, blockIdx.x / ns, seg, chunk);
  const int rows = seg_rows(g.p, seg);
  const int c_lo = cs * CSW;
  load_tables(g.lz, seg, 1.f / (float)rows, c_lo, min(C, c_lo + CSW), ax, nullptr, nullptr, nullptr);
  __syncthreads();
  if (rr >= geo.R) return;
  const int off = g.p.row_off[seg];
  const int m_begin = off + chunk * geo.CH, m_end = min(off + rows, m_begin + geo.CH);
  const int hw = g.p.H[seg] * g.p.W[seg];
  const int NV = C / 8;
  T* OUT = (T*)g.dx;
#pragma unroll
  for (int v = 0; v < RVPT; ++v) {
    const int cv = c_lo / 8 + tv + v * geo.TPR;
    if (!(v < geo.VPT && cv < NV)) continue;
    const int c = cv * 8;
    float2 a8[8];  // the 8 channels' affine in registers
#pragma unroll
    for (int j = 0; j < 8; ++j) a8[j] = ax[c + j];
    for (int m = m_begin + rr; m < m_end; m += EUR * geo.R) {
      float x[EUR][8], gt[EUR][8];
#pragma unroll
      for (int u = 0; u < EUR; ++u) {
        const int mu = min(m + u * geo.R, m_end - 1);
        ld8((const T*)g.lz.x + (size_t)mu * g.lz.ld + c, x[u]);
        if (GATE) ld8(g.lz.gate + (size_t)((mu - off) / hw) * C + c, gt[u]);
      }
#pragma unroll
      for (int u = 0; u < EUR; ++u) {
        const int mu = m + u * geo.R;
        if (mu >= m_end) break;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          x[u][j] = lazy_apply(x[u][j], a8[j], ACT);
          if (GATE) x[u][j] *= gt[u][j];
        }
        st8(OUT + (size_t)mu * C + c, x[u]);
      }
    }
  }
}

// Keras BatchNormalization moving statistics: m -= (m - batch) * (1 - momentum), with the
// Bessel-corrected batch variance that FusedBatchNormV3 returns in training mode.
// `skip` (nullable): edet_opt_apply's scalars[6]; a step the optimizer skipped as non-finite
// (sched.skip_nonfinite) leaves the moving statistics unchanged too (its batch statistics
// are as suspect as its gradient)
__global__ void k_bn_update(int64_t n, const double* sum, const double* sq, const float* count,
                            float momentum, const float* skip, float* mmean, float* mvar) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (skip && *skip != 0.f) return;
  const double cnt = count[i];
  const double mean = stat_get(sum, (int)i) / cnt;
  const double var = fmax(stat_get(sq, (int)i) / cnt - mean * mean, 0.0);
  const float unb = (float)(var * cnt / fmax(cnt - 1.0, 1.0));
  mmean[i] -= (mmean[i] - (float)mean) * (1.f - momentum);
  mvar[i] -= (mvar[i] - unb) * (1.f - momentum);
}

__global__ void k_bn_infer_stats(int64_t n, const float* mm, const float* mv, const float* count, double* sum,
                                 double* sq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double c = count[i], m = mm[i];
  sum[stat_idx((int)i, 0)] = m * c;  // replica 0; the other three stay zero
  sq[stat_idx((int)i, 0)] = ((double)mv[i] + m * m) * c;
}

static int lazy_checks(const edet_lazy* x, const edet_pyramid* p, int C) {
  EDET_REQUIRE(x && p && x->x, "lazy: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0 && C <= 8 * 256 * RVPT, "lazy: need C%%8==0, ld%%8==0, C<=4096 (C=%d ld=%d)", C, x->ld);
  EDET_REQUIRE(p->nseg >= 1 && p->nseg <= EDET_MAX_SEG, "lazy: bad pyramid");
  EDET_REQUIRE(x->gate == nullptr || p->nseg == 1, "lazy: gate needs one segment");
  return EDET_OK;
}

template <typename T, int F = 0>
static void launch_reduce(int f, dim3 grid, dim3 block, size_t lds, hipStream_t s, const LArgs& g, int nb) {
  if constexpr (F < 32) {
    if (f == F) EDET_LAUNCH((k_lazy_bwd_reduce<T, F>), grid, block, lds, s, g, nb);
    else launch_reduce<T, F + 2>(f, grid, block, lds, s, g, nb);
  }
}
template <typename T, bool NT = false, int F = 0>
static void launch_apply(int f, dim3 grid, dim3 block, size_t lds, hipStream_t s, const LArgs& g, int nb) {
  if constexpr (F < 64) {
    if (f == F) EDET_LAUNCH((k_lazy_bwd_apply<T, F, NT>), grid, block, lds, s, g, nb);
    else launch_apply<T, NT, F + 1>(f, grid, block, lds, s, g, nb);
  }
}

}  // namespace edet

using namespace edet;

extern "C" {

static dim3 row_block(const RowGeom& geo) { return dim3(geo.TPR * geo.R); }

int edet_lazy_bwd_reduce(int dtype, const edet_lazy* x, const edet_pyramid* p, int C,
                         const void* dv, const float* dv_scale, const float* dsq,
                         const edet_bngrad64* acc, edet_stream_t stream) {
  int rc = lazy_checks(x, p, C);
  if (rc) return rc;
  EDET_REQUIRE(dv && acc && x->bn.enabled, "lazy_bwd_reduce: needs dv, acc and an enabled BN");
  EDET_REQUIRE(dsq == nullptr || p->nseg == 1, "lazy_bwd_reduce: dsq needs one segment");
  LArgs g{};
  g.lz = *x; g.p = *p; g.acc = *acc; g.dv = dv; g.dv_scale = dv_scale; g.dsq = dsq; g.C = C;
  // Every block flushes 2C fp64 atomics to the same addresses, which serialise (~20 ns per
  // block and address): long chunks and at most 512 persistent blocks measured best (r01g,
  // four rows per trip: 256 / 384 / 512 / 768 / 1024 / 2048 -> 1.49 / 1.45 / 1.43 / 1.51 /
  // 1.51 / 1.52 ms/step)
  // (scripts/row_probe.py: -20..-30 % on the C >= 240 and C = 16 layers, equal elsewhere).
  // 32 passes for the wide layers (kbench sweep, round 2: 524288 x 144 60 -> 52 us, 32768 x 480
  // 24 -> 21 us)
  // Round 3 (profiles/r03ad_bn_plan_sweep.txt): short rows want shorter chunks, 8 passes for
  // C <= 64 and 16 for C >= 144 at M <= 8192 (8192 x 192: 36.2 -> 29.9 us per step, the BiFPN
  // 2048 x 64: 43.3 -> 37.1), and the narrow C <= 24 tensors 256 blocks (2M x 16: 31.5 -> 28.0)
  // Round 6 (replicated statistics, profiles/r06/r06v_plan_resweep.txt): the single tensors up to
  // 32768 rows want 8 passes (32768 x 64: 57.0 -> 48.2 us, 8192 x 192: 28.8 -> 23.5, 32768 x 112:
  // 22.6 -> 20.6), and the narrow C <= 24 tensors up to 524288 rows 1024 blocks (28.1 -> 25.7)
  const int M = pyr_valid_rows(*p);
  int passes = C >= 144 && p->nseg == 1 ? 32 : 16;
  if (M <= 8192 && C < 1024) passes = C <= 64 ? 8 : 16;  // D4's 8192 x 2688 keeps 32 (46.6 vs 64.0 us)
  if (p->nseg == 1 && M <= 32768 && C < 1024) passes = 8;
  g.geo = row_geom(C, dev_knob(10) > 0 ? dev_knob(10) : passes);
  const int nb = total_chunks(*p, g.geo.CH);
  const size_t lds = 2 * C * sizeof(float2) + 2 * (size_t)g.geo.R * C * sizeof(float);
  EDET_DTYPE_DISPATCH(dtype, T, {
    // persistent blocks (r01h sweep: 1.51 -> 1.43 ms/step against 1024)
    const int rcap = dev_knob(11) > 0 ? dev_knob(11) : (C <= 24 ? (M <= 524288 ? 1024 : 256) : 512);
    const int grid = nb < rcap ? nb : rcap;
    const int f = (x->act ? AF_ACT : 0) | (x->gate ? AF_GATE : 0) | (dsq ? AF_DSQ : 0) | (dv_scale ? AF_DVS : 0);
    if (nb) launch_reduce<T>(f, dim3(grid), row_block(g.geo), lds, (hipStream_t)stream, g, nb);
    return check_launch("edet lazy_bwd_reduce");
  });
}

int edet_lazy_bwd_apply(int dtype, const edet_lazy* x, const edet_pyramid* p, int C,
                        const void* dv, const float* dv_scale, const float* dsq,
                        const edet_bngrad64* acc, const edet_segout* grads, void* dx,
                        int accumulate, edet_stream_t stream) {
  int rc = lazy_checks(x, p, C);
  if (rc) return rc;
  EDET_REQUIRE(dv && dx, "lazy_bwd_apply: null dv/dx");
  EDET_REQUIRE(!x->bn.enabled || acc, "lazy_bwd_apply: BN needs the reduced fp64 sums");
  EDET_REQUIRE(dsq == nullptr || p->nseg == 1, "lazy_bwd_apply: dsq needs one segment");
  LArgs g{};
  g.lz = *x; g.p = *p; g.dv = dv; g.dx = dx; g.dv_scale = dv_scale;
  if (acc) g.acc = *acc;
  if (grads && x->bn.enabled) { g.grads = *grads; g.has_grads = 1; }
  g.dsq = dsq; g.C = C; g.accumulate = accumulate;
  // short chunks (persistent grid): 2.25 -> 2.21 ms/step against 8-16 passes; 8 from C = 480 up
  // (fewer, longer-lived blocks: M = 8192, C = 1152: 25 -> 21 us; kbench sweep, round 2)
  // Round 3 (profiles/r03ad_bn_plan_sweep.txt): the BiFPN C = 64 levels at M <= 8192 2 passes
  // (8192 x 64 +sw: 26.5 -> 22.8 us per step), SE-gated 96 <= C < 480 8 (524288 x 96: 63.8 ->
  // 59.3, 32768 x 240: 15.0 -> 12.9), C >= 672 over M >= 32768 16 (32768 x 672: 84.8 -> 79.8),
  // C < 1024 over M <= 8192 4 (8192 x 672: 13.9 -> 12.4)
  const int M = pyr_valid_rows(*p);
  int passes = C >= 480 ? 8 : 4;
  if (C <= 64 && M <= 8192) passes = 2;
  else if (x->gate && C >= 96 && C < 480) passes = 8;
  else if (C >= 672 && M >= 32768) passes = 16;
  else if (C >= 480 && C <= 672 && M <= 8192) passes = 4;  // not D4's 8192 x 960 (15.3 vs 17.6 us)
  // round 6 (profiles/r06/r06ae_apply_materialize_sweep.txt): 8 passes for the ungated mid-width
  // tensors up to 131072 rows (131072 x 240: 68.3 -> 64.5 us, 32768 x 112: 27.6 -> 22.2) and the
  // C = 64 head pyramids (174592 x 64: 96.0 -> 89.9)
  if (!x->gate && C >= 96 && C < 480 && M > 8192 && M <= 131072) passes = 8;
  else if (p->nseg > 1 && C <= 64) passes = 8;
  g.geo = row_geom(C, dev_knob(8) > 0 ? dev_knob(8) : passes);
  g.cslices = 1;
  // wide rows over few of them (C >= 1024, M <= 16384: the 16^2 stage): 64-channel slices, 32 rows
  // per pass, 4 passes per chunk (development slot 55: 1 = always from C >= 256, 2 = never;
  // slot 56: passes)
  const bool sliced = dev_knob(55) == 1 ? C >= 256 : (dev_knob(55) != 2 && C >= 1024 && M <= 16384);
  if (sliced) {
    g.geo.TPR = 8; g.geo.R = 32; g.geo.VPT = 1;
    g.geo.CH = 32 * (dev_knob(56) > 0 ? dev_knob(56) : 4);
    g.cslices = cdiv(C / 8, 8);
  }
  const int nb = total_chunks(*p, g.geo.CH);
  const size_t lds = 3 * C * sizeof(float2);
  EDET_DTYPE_DISPATCH(dtype, T, {
    // resident blocks per launch: 512 for the long ungated tensors (M >= 524288, C >= 96: 2M x 96
    // 235.6 -> 222.9 us, 524288 x 144 180.5 -> 176.4, r05i sweep), 2048 elsewhere
    const int gcap = dev_knob(9) > 0 ? dev_knob(9) : ((M >= 524288 && C >= 96 && !x->gate) ? 512 : 2048);
    const int grid = nb * g.cslices > gcap ? gcap : nb * g.cslices;
    const int f = (x->bn.enabled ? AF_BN : 0) | (x->act ? AF_ACT : 0) | (x->gate ? AF_GATE : 0) | (dsq ? AF_DSQ : 0) |
                  (dv_scale ? AF_DVS : 0) | (accumulate ? AF_ACC : 0);
    // nontemporal row loads / stores over >= 524288 rows (2M x 96: 222 -> 215 us, 524288 x 144:
    // 87 -> 83; on every apply they cost the small ones their cache hits, r05an).  Development
    // slot 53: 1 = from slot 54's row count, 2 = never
    const long nt_rows = dev_knob(53) == 1 ? dev_knob(54) : 524288;
    if (nb && sizeof(T) == 2 && !accumulate && dev_knob(53) != 2 && M >= nt_rows) {
      launch_apply<T, true>(f, dim3(grid), row_block(g.geo), lds, (hipStream_t)stream, g, nb);
      return check_launch("edet lazy_bwd_apply");
    }
    if (nb) launch_apply<T>(f, dim3(grid), row_block(g.geo), lds, (hipStream_t)stream, g, nb);
    return check_launch("edet lazy_bwd_apply");
  });
}

// the per-image reductions (SE squeeze, SE-fused BN reduce) shorten their chunks until a launch
// holds at least this many blocks (two per CU)
constexpr long FILL_BLOCKS = 512;

static int img_reduce(int dtype, bool gategrad, const edet_lazy* x, int B, int HW, int C,
                      const void* dv, double* out64, hipStream_t s) {
  EDET_REQUIRE(x && out64 && x->x && (!gategrad || dv), "se reduce: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0 && C <= 8 * 256 * RVPT, "se reduce: need C%%8==0");
  LArgs g{};
  g.lz = *x; g.lz.gate = nullptr;  // the pre-gate value
  g.p.nseg = 1; g.p.batch = B; g.p.row_off[0] = 0; g.p.H[0] = HW; g.p.W[0] = 1;
  g.dv = dv; g.out64 = out64; g.C = C; g.hw = HW;
  // long chunks: each block ends in C fp64 atomics; round 6: halved (down to 4 passes) while the
  // launch would hold fewer than FILL_BLOCKS blocks (the 32^2 / 64^2 stages ran 128-320 blocks)
  int passes = dev_knob(44) > 0 ? dev_knob(44) : 16;
  if (dev_knob(44) == 0)
    while (passes > 4 && (long)B * cdiv(HW, row_geom(C, passes).CH) < FILL_BLOCKS) passes /= 2;
  g.geo = row_geom(C, passes);
  g.cslices = 1;
  // C >= 480 over H*W <= 4096: a block per (image, 64-channel slice) over the whole image, as
  // edet_gate_bn_reduce (development slot 46 = 2: off)
  if (dev_knob(46) != 2 && C >= 480 && C <= 2048 && HW <= 4096) {
    g.geo.TPR = 8; g.geo.R = 32; g.geo.VPT = 1; g.geo.CH = HW;
    g.cslices = cdiv(C / 8, 8);
  }
  g.chunks_per_img = cdiv(HW, g.geo.CH);
  const int nb = B * g.chunks_per_img * g.cslices;
  const size_t lds = C * sizeof(float2) + (size_t)g.geo.R * (g.cslices > 1 ? g.geo.TPR * 8 : C) * sizeof(float);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (gategrad && x->act) EDET_LAUNCH((k_img_reduce<T, true, true>), dim3(nb), row_block(g.geo), lds, s, g);
    else if (gategrad) EDET_LAUNCH((k_img_reduce<T, true, false>), dim3(nb), row_block(g.geo), lds, s, g);
    else if (x->act) EDET_LAUNCH((k_img_reduce<T, false, true>), dim3(nb), row_block(g.geo), lds, s, g);
    else EDET_LAUNCH((k_img_reduce<T, false, false>), dim3(nb), row_block(g.geo), lds, s, g);
    return check_launch("edet se reduce");
  });
}

int edet_se_squeeze(int dtype, const edet_lazy* x, int B, int HW, int C, double* s,
                    edet_stream_t stream) {
  return img_reduce(dtype, false, x, B, HW, C, nullptr, s, (hipStream_t)stream);
}

int edet_gate_grad(int dtype, const edet_lazy* x, int B, int HW, int C, const void* dv,
                   double* dgate, edet_stream_t stream) {
  return img_reduce(dtype, true, x, B, HW, C, dv, dgate, (hipStream_t)stream);
}

int edet_gate_bn_reduce(int dtype, const edet_lazy* x, int B, int HW, int C, const void* dv,
                        double* sums5, edet_stream_t stream) {
  EDET_REQUIRE(x && x->x && dv && sums5, "gate_bn_reduce: null argument");
  EDET_REQUIRE(x->bn.enabled && x->act == EDET_ACT_SWISH, "gate_bn_reduce: needs bn + swish");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0 && C <= 2048, "gate_bn_reduce: need C%%8==0, C<=2048");
  LArgs g{};
  g.lz = *x; g.lz.gate = nullptr;
  g.p.nseg = 1; g.p.batch = B; g.p.row_off[0] = 0; g.p.H[0] = HW; g.p.W[0] = 1;
  g.dv = dv; g.out64 = sums5; g.C = C; g.hw = HW;
  // long chunks: every block ends in 5C fp64 atomics (0.69 -> 0.54 ms/step at 16 passes vs ~8;
  // 32 passes: 0.58 in round 1, 0.45 against 0.48 in the round-2 sweep after the table hoists)
  // (round 6: halved, down to 4 passes, while the launch would hold fewer than FILL_BLOCKS
  // blocks: 32768 x 240 ran 128 blocks)
  int passes = dev_knob(12) > 0 ? dev_knob(12) : 32;
  if (dev_knob(12) == 0)
    while (passes > 4 && (long)B * cdiv(HW, row_geom(C, passes).CH) < FILL_BLOCKS) passes /= 2;
  g.geo = row_geom(C, passes);
  g.cslices = 1;
  // wide rows over short images (C >= 480, H*W <= 4096: the 16^2 / 32^2 / 64^2 stages): a block
  // per (image, 64-channel slice) walks the whole image, 32 rows per pass, and owns its outputs
  // (development slot 46: 1 = always, 2 = never)
  const bool sliced = dev_knob(46) == 1 || (dev_knob(46) != 2 && C >= 480 && HW <= 4096);
  if (sliced) {
    const int tpr = dev_knob(47) > 0 ? dev_knob(47) : 8;  // development slot 47: vectors per slice
    g.geo.TPR = tpr; g.geo.R = 256 / tpr; g.geo.VPT = 1; g.geo.CH = HW;
    g.cslices = cdiv(C / 8, tpr);
  }
  g.chunks_per_img = cdiv(HW, g.geo.CH);
  const int nb = B * g.chunks_per_img * g.cslices;
  const size_t lds = 2 * C * sizeof(float2) + (size_t)g.geo.R * g.geo.TPR * 8 * sizeof(float);
  EDET_DTYPE_DISPATCH(dtype, T, {
    EDET_LAUNCH(k_gate_bn_reduce<T>, dim3(nb), row_block(g.geo), lds, (hipStream_t)stream, g);
    return check_launch("edet gate_bn_reduce");
  });
}

int edet_se_bn_combine(int B, int C, const float* gate, const float* dsq, const double* sums5,
                       const edet_bngrad64* acc, edet_stream_t stream) {
  EDET_REQUIRE(gate && dsq && sums5 && acc && acc->dgamma[0] && acc->dbeta[0], "se_bn_combine: null argument");
  EDET_LAUNCH(k_se_bn_combine, dim3(cdiv(C, 8)), dim3(256), 0, (hipStream_t)stream, B, C, gate, dsq, sums5,
                     acc->dgamma[0], acc->dbeta[0]);
  return check_launch("edet se_bn_combine");
}

int edet_se_fwd(int B, int C, int R, const double* s, const float* w1, const float* b1,
                const float* w2, const float* b2, float* z1, float* gate, edet_stream_t stream) {
  EDET_REQUIRE(s && w1 && b1 && w2 && b2 && z1 && gate && B > 0 && C > 0 && R > 0,
               "se_fwd: bad argument");
  hipStream_t st = (hipStream_t)stream;
  EDET_LAUNCH(k_se_reduce_c, dim3(cdiv(B * R, 4)), dim3(256), 0, st, B, C, R, s, w1, b1, z1);
  EDET_LAUNCH(k_se_excite, dim3(cdiv(B * C, 256)), dim3(256), 0, st, B, C, R, z1, w2, b2, gate);
  return check_launch("edet se_fwd");
}

int edet_se_bwd_bn(int B, int C, int R, int HW, const double* s, const float* z1,
                   const float* gate, const double* dgate, const float* w1, const float* w2,
                   float* dw1, float* db1, float* dw2, float* db2, float* dsq, float* dz1,
                   const double* sums5, const edet_bngrad64* acc, edet_stream_t stream) {
  EDET_REQUIRE(s && z1 && gate && dgate && w1 && w2 && dw1 && db1 && dw2 && db2 && dsq && dz1 && sums5 && acc &&
                   acc->dgamma[0] && acc->dbeta[0],
               "se_bwd_bn: null argument");
  hipStream_t st = (hipStream_t)stream;
  EDET_LAUNCH(k_se_dz1, dim3(cdiv(B * R, 4)), dim3(256), 0, st, B, C, R, z1, gate, dgate, w2, dz1);
  const int nA = se_wgrad_blocks(C, R), nB = cdiv(std::max(B * C, std::max(C, R)), 256);
  EDET_LAUNCH(k_se_wgrad_bn, dim3(nA + nB + cdiv(C, 8)), dim3(256), 0, st, B, C, R, HW, nA, nA + nB, s, z1, gate,
              dgate, dz1, w1, dw1, db1, dw2, db2, dsq, sums5, acc->dgamma[0], acc->dbeta[0]);
  return check_launch("edet se_bwd_bn");
}

int edet_se_bwd(int B, int C, int R, int HW, const double* s, const float* z1,
                const float* gate, const double* dgate, const float* w1, const float* w2,
                float* dw1, float* db1, float* dw2, float* db2, float* dsq, float* dz1,
                edet_stream_t stream) {
  EDET_REQUIRE(s && z1 && gate && dgate && w1 && w2 && dw1 && db1 && dw2 && db2 && dsq && dz1,
               "se_bwd: null argument");
  hipStream_t st = (hipStream_t)stream;
  EDET_LAUNCH(k_se_dz1, dim3(cdiv(B * R, 4)), dim3(256), 0, st, B, C, R, z1, gate, dgate, w2, dz1);
  const int nA = se_wgrad_blocks(C, R), nB = cdiv(std::max(B * C, std::max(C, R)), 256);
  EDET_LAUNCH(k_se_wgrad, dim3(nA + nB), dim3(256), 0, st, B, C, R, HW, nA, s, z1, gate, dgate, dz1, w1,
                     dw1, db1, dw2, db2, dsq);
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
  g.geo = row_geom(C);
  const int nb = total_chunks(*p, g.geo.CH);
  const size_t lds = 2 * C * sizeof(float2);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_residual<T>, dim3(nb), row_block(g.geo), lds, (hipStream_t)stream, g);
    return check_launch("edet residual");
  });
}

int edet_lazy_materialize(int dtype, const edet_lazy* x, const edet_pyramid* p, int C, void* out,
                          edet_stream_t stream) {
  int rc = lazy_checks(x, p, C);
  if (rc) return rc;
  EDET_REQUIRE(out, "lazy_materialize: null out");
  LArgs g{};
  g.lz = *x; g.p = *p; g.dx = out; g.C = C;
  // 0.60 -> 0.56 ms/step against ~8 passes; 8 for C >= 1024 (M = 8192, C = 1152: 15 -> 13 us)
  // and 8 for 144 <= C over 32768 <= M <= 131072 (32768 x 480: 42.4 -> 40.5 us per step,
  // profiles/r03ad_bn_plan_sweep.txt)
  const int M = pyr_valid_rows(*p);
  // (round 6, r06ae: 8 also for C >= 144 over >= 524288 rows, 524288 x 144: 58.5 -> 55.8 us)
  const bool mid = C >= 144 && M >= 32768 && (M <= 131072 || M >= 524288);
  g.geo = row_geom(C, dev_knob(13) > 0 ? dev_knob(13) : (C >= 1024 || mid ? 8 : 4));
  g.cslices = 1;
  // C >= 1024 over M <= 16384: 64-channel slices, 32 rows per pass (as edet_lazy_bwd_apply;
  // development slot 57: 1 = from C >= 256, 2 = never; slot 58: passes)
  if (dev_knob(57) == 1 ? C >= 256 : (dev_knob(57) != 2 && C >= 1024 && M <= 16384)) {
    g.geo.TPR = 8; g.geo.R = 32; g.geo.VPT = 1;
    g.geo.CH = 32 * (dev_knob(58) > 0 ? dev_knob(58) : 2);
    g.cslices = cdiv(C / 8, 8);
  }
  const int nb = total_chunks(*p, g.geo.CH) * g.cslices;
  const size_t lds = C * sizeof(float2);
  EDET_DTYPE_DISPATCH(dtype, T, {
    const hipStream_t st = (hipStream_t)stream;
    if (nb && x->act && x->gate) EDET_LAUNCH((k_materialize<T, true, true>), dim3(nb), row_block(g.geo), lds, st, g);
    else if (nb && x->act) EDET_LAUNCH((k_materialize<T, true, false>), dim3(nb), row_block(g.geo), lds, st, g);
    else if (nb && x->gate) EDET_LAUNCH((k_materialize<T, false, true>), dim3(nb), row_block(g.geo), lds, st, g);
    else if (nb) EDET_LAUNCH((k_materialize<T, false, false>), dim3(nb), row_block(g.geo), lds, st, g);
    return check_launch("edet lazy_materialize");
  });
}

int edet_bn_inference_stats(int64_t n, const float* mmean, const float* mvar, const float* count,
                            double* sum, double* sq, edet_stream_t stream) {
  EDET_REQUIRE(mmean && mvar && count && sum && sq, "bn_inference_stats: null argument");
  if (n <= 0) return EDET_OK;
  EDET_LAUNCH(k_bn_infer_stats, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     mmean, mvar, count, sum, sq);
  return check_launch("edet bn_inference_stats");
}

int edet_bn_update_moving(int64_t n, const double* sum, const double* sq, const float* count,
                          float momentum, const float* skip, float* mmean, float* mvar,
                          edet_stream_t stream) {
  EDET_REQUIRE(sum && sq && count && mmean && mvar, "bn_update_moving: null argument");
  if (n <= 0) return EDET_OK;
  EDET_LAUNCH(k_bn_update, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     n, sum, sq, count, momentum, skip, mmean, mvar);
  return check_launch("edet bn_update_moving");
}

}  // extern "C"
