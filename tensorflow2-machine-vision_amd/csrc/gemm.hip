// Pointwise (1x1) convolution as MFMA GEMMs over NHWC rows.
//
//   forward : y[m][n]  = sum_k v(a)[m][k] * wt[n][k] (+ bias[n]); v(.) = lazy BN/swish/SE-gate
//             applied while staging A into LDS; epilogue accumulates per-segment BN
//             statistics (sum, sum of squares) of y -> the consumer normalises on load.
//   dgrad   : dx[m][k] = sum_n dy[m][n] * wt[n][k]
//   wgrad   : dwt[n][k] += sum_m dy[m][n] * v(a)[m][k], dbias[n] += sum_m dy[m][n]
//
// Replaces the Conv2D 1x1 layers of layers/mb_conv_block.py:62-69,105-112 (expand/project),
// layers/resample_feature_map.py:24-27 and the pointwise half of every SeparableConv2D
// (layers/bifpn.py:16-21, layers/class_net.py:54-76, layers/box_net.py:49-78).
//
// Tiling: 256 threads = 4 waves in a 2x2 arrangement, BM x BN output tile, K staged in
// chunks of 32 through LDS (register-staged so the lazy transform can be applied), bf16
// math on v_mfma_f32_16x16x32_bf16, fp32 math on v_mfma_f32_16x16x4_f32 (exact f32).
#include "common.hpp"

namespace edet {

constexpr int GBK = 32;
constexpr int GLDK = GBK + 8;  // padded LDS row (elements): 80 B bf16 / 160 B fp32

struct GemmArgs {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  edet_lazy lz;
  edet_pyramid pyr;
  edet_segout stats;
  int lda, ldb, ldc, M, K, N;
  int accumulate, has_stats, ntm, ntn;
};

// raw copy of 8 elements global -> LDS with zero fill past n valid
template <typename T>
__device__ __forceinline__ void cp8(T* dst, const T* src, int n) {
  if (n >= 8) {
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    } else {
      reinterpret_cast<float4*>(dst)[0] = reinterpret_cast<const float4*>(src)[0];
      reinterpret_cast<float4*>(dst)[1] = reinterpret_cast<const float4*>(src)[1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[i] = (i < n) ? src[i] : T(0);
  }
}
template <typename T>
__device__ __forceinline__ void zero8(T* dst) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(dst) = make_uint4(0, 0, 0, 0);
  } else {
    reinterpret_cast<float4*>(dst)[0] = make_float4(0, 0, 0, 0);
    reinterpret_cast<float4*>(dst)[1] = make_float4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ bf16x8_t lds_frag_bf16(const uint16_t* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return __builtin_bit_cast(bf16x8_t, v);
}

template <typename T, int BM, int BN, bool BT, bool LAZY>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) T As[BM * GLDK];
  __shared__ __attribute__((aligned(16))) T Bs[BN * GLDK];
  __shared__ float red[2][BN];
  extern __shared__ float2 xf[];  // [K] lazy affine per input channel (LAZY only)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = t / g.ntn, tn = t - tm * g.ntn;
  const int row0 = tm * BM, col0 = tn * BN;

  int seg = 0;
  if (LAZY || g.has_stats) seg = seg_of_row(g.pyr, row0);
  const int seg_off = g.pyr.row_off[seg];
  const int seg_end = seg_off + seg_rows(g.pyr, seg);
  const int hw = g.pyr.H[seg] * g.pyr.W[seg];

  if constexpr (LAZY) {
    const float inv = 1.f / (float)seg_rows(g.pyr, seg);
    for (int k = tid; k < g.K; k += 256) xf[k] = bn_affine(g.lz.bn, seg, k, inv);
  }
  if (g.has_stats)
    for (int i = tid; i < 2 * BN; i += 256) (&red[0][0])[i] = 0.f;
  __syncthreads();

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const T* A = (const T*)g.a;
  const T* B = (const T*)g.b;

  for (int k0 = 0; k0 < g.K; k0 += GBK) {
    // ---- stage A (BM x 32): lazy transform applied here
    for (int v = tid; v < BM * (GBK / 8); v += 256) {
      const int r = v >> 2, kv = (v & 3) * 8;
      const int grow = row0 + r, gk = k0 + kv, nk = g.K - gk;
      T* dst = &As[r * GLDK + kv];
      if (grow < g.M && nk > 0) {
        if constexpr (LAZY) {
          float vals[8];
          ld8m(A + (size_t)grow * g.lda + gk, nk, vals);
          const float* gp = g.lz.gate ? g.lz.gate + (size_t)((grow - seg_off) / hw) * g.K : nullptr;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (j < nk) {
              float2 af = xf[gk + j];
              float u = lazy_apply(vals[j], af, g.lz.act);
              if (gp) u *= gp[gk + j];
              vals[j] = u;
            }
          }
          st8(dst, vals);
        } else {
          cp8(dst, A + (size_t)grow * g.lda + gk, nk);
        }
      } else {
        zero8(dst);
      }
    }
    // ---- stage B as Bs[n][k]
    if constexpr (BT) {  // B is [N][ldb], k contiguous
      for (int v = tid; v < BN * (GBK / 8); v += 256) {
        const int n = v >> 2, kv = (v & 3) * 8;
        const int gn = col0 + n, gk = k0 + kv, nk = g.K - gk;
        T* dst = &Bs[n * GLDK + kv];
        if (gn < g.N && nk > 0) cp8(dst, B + (size_t)gn * g.ldb + gk, nk);
        else zero8(dst);
      }
    } else {  // B is [K][ldb], n contiguous: transpose into LDS
      for (int v = tid; v < GBK * (BN / 8); v += 256) {
        const int kk = v / (BN / 8), nv = (v - kk * (BN / 8)) * 8;
        const int gk = k0 + kk, gn = col0 + nv, nn = g.N - gn;
        float vals[8];
        if (gk < g.K && nn > 0) ld8m(B + (size_t)gk * g.ldb + gn, nn, vals);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) vals[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) Bs[(nv + j) * GLDK + kk] = from_f<T>(vals[j]);
      }
    }
    __syncthreads();

    if constexpr (sizeof(T) == 2) {
      bf16x8_t af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = lds_frag_bf16(&As[(wm * WM + i * 16 + (lane & 15)) * GLDK + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = lds_frag_bf16(&Bs[(wn * WN + j * 16 + (lane & 15)) * GLDK + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < GBK / 4; ++s) {
        float af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = As[(wm * WM + i * 16 + (lane & 15)) * GLDK + 4 * s + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = Bs[(wn * WN + j * 16 + (lane & 15)) * GLDK + 4 * s + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- epilogue: bias, store (optionally accumulate), BN statistics
  T* C = (T*)g.c;
  float ssum[FN], ssq[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { ssum[j] = 0.f; ssq[j] = 0.f; }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = col0 + wn * WN + j * 16 + (lane & 15);
    const float bv = (g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        const float v = acc[i][j][r] + bv;
        if (row < g.M && col < g.N) {
          T* p = C + (size_t)row * g.ldc + col;
          *p = from_f<T>(g.accumulate ? to_f<T>(*p) + v : v);
          if (row < seg_end) { ssum[j] += v; ssq[j] += v * v; }
        }
      }
    }
  }
  if (g.has_stats) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = ssum[j], q = ssq[j];
      s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
      q += __shfl_xor(q, 16, 64); q += __shfl_xor(q, 32, 64);
      if (lane < 16) {
        atomicAdd(&red[0][wn * WN + j * 16 + lane], s);
        atomicAdd(&red[1][wn * WN + j * 16 + lane], q);
      }
    }
    __syncthreads();
    for (int i = tid; i < BN; i += 256) {
      const int col = col0 + i;
      if (col < g.N) {
        atomicAdd(g.stats.a[seg] + col, red[0][i]);
        atomicAdd(g.stats.b[seg] + col, red[1][i]);
      }
    }
  }
}

// ------------------------------------------------------------------ weight gradient
struct WgradArgs {
  const void* a;
  const void* dy;
  float* dw;
  float* db;
  edet_lazy lz;
  edet_pyramid pyr;
  int lda, lddy, M, K, N;
  int ntn, ntk, rows_per;
};

template <typename T, bool LAZY>
__global__ __launch_bounds__(256) void k_wgrad(WgradArgs g) {
  constexpr int TN = 64, TK = 64, BMM = 32, LDM = BMM + 8;
  __shared__ __attribute__((aligned(16))) T Ds[TN * LDM];  // dy^T tile  [n][m]
  __shared__ __attribute__((aligned(16))) T Xs[TK * LDM];  // v(a)^T tile [k][m]
  __shared__ float2 xf[TK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int ntiles = g.ntn * g.ntk;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / ntiles, tile = lid - split * ntiles;
  const int tn = tile / g.ntk, tk = tile - tn * g.ntk;
  const int n0 = tn * TN, kk0 = tk * TK;
  const int m_begin = split * g.rows_per;
  const int m_end = min(g.M, m_begin + g.rows_per);
  const bool do_db = (g.db != nullptr) && tk == 0;
  const T* DY = (const T*)g.dy;
  const T* A = (const T*)g.a;

  floatx4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  int cur_seg = -1;

  for (int m0 = m_begin; m0 < m_end; m0 += BMM) {
    const int seg = seg_of_row(g.pyr, m0);
    __syncthreads();
    if (LAZY && seg != cur_seg) {
      if (tid < TK) {
        const int k = kk0 + tid;
        xf[tid] = (k < g.K) ? bn_affine(g.lz.bn, seg, k, 1.f / (float)seg_rows(g.pyr, seg))
                            : make_float2(1.f, 0.f);
      }
      __syncthreads();
    }
    cur_seg = seg;
    const int seg_off = g.pyr.row_off[seg];
    const int seg_end = seg_off + seg_rows(g.pyr, seg);
    const int hw = g.pyr.H[seg] * g.pyr.W[seg];
    {
      const int m = tid >> 3, nv = (tid & 7) * 8;
      const int row = m0 + m, gn = n0 + nv, nn = g.N - gn;
      float vals[8];
      if (row < m_end && row < seg_end && nn > 0) ld8m(DY + (size_t)row * g.lddy + gn, nn, vals);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) Ds[(nv + j) * LDM + m] = from_f<T>(vals[j]);
    }
    {
      const int m = tid >> 3, kv = (tid & 7) * 8;
      const int row = m0 + m, gk = kk0 + kv, nk = g.K - gk;
      float vals[8];
      if (row < m_end && row < seg_end && nk > 0) {
        ld8m(A + (size_t)row * g.lda + gk, nk, vals);
        if constexpr (LAZY) {
          const float* gp = g.lz.gate ? g.lz.gate + (size_t)((row - seg_off) / hw) * g.K : nullptr;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (j < nk) {
              float u = lazy_apply(vals[j], xf[kv + j], g.lz.act);
              if (gp) u *= gp[gk + j];
              vals[j] = u;
            }
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) Xs[(kv + j) * LDM + m] = from_f<T>(vals[j]);
    }
    __syncthreads();
    if (do_db && tid < TN) {
      float s = 0.f;
#pragma unroll 8
      for (int m = 0; m < BMM; ++m) s += to_f<T>(Ds[tid * LDM + m]);
      dbacc += s;
    }
    if constexpr (sizeof(T) == 2) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = lds_frag_bf16(&Ds[(wn * 32 + i * 16 + (lane & 15)) * LDM + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = lds_frag_bf16(&Xs[(wk * 32 + j * 16 + (lane & 15)) * LDM + 8 * (lane >> 4)]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < BMM / 4; ++s) {
        float af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = Ds[(wn * 32 + i * 16 + (lane & 15)) * LDM + 4 * s + (lane >> 4)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = Xs[(wk * 32 + j * 16 + (lane & 15)) * LDM + 4 * s + (lane >> 4)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int k = kk0 + wk * 32 + j * 16 + (lane & 15);
        if (n < g.N && k < g.K) atomicAdd(g.dw + (size_t)n * g.K + k, acc[i][j][r]);
      }
  if (do_db && tid < TN && n0 + tid < g.N) atomicAdd(g.db + n0 + tid, dbacc);
}

// ------------------------------------------------------------------ launch helpers
template <typename T, int BM, int BN, bool BT, bool LAZY>
static int launch_gemm(GemmArgs g, hipStream_t s) {
  g.ntm = cdiv(g.M, BM);
  g.ntn = cdiv(g.N, BN);
  const int nwg = g.ntm * g.ntn;
  if (nwg == 0) return EDET_OK;
  const size_t dyn = LAZY ? (size_t)g.K * sizeof(float2) : 0;
  hipLaunchKernelGGL((k_gemm<T, BM, BN, BT, LAZY>), dim3(nwg), dim3(256), dyn, s, g);
  return check_launch("edet gemm");
}

static int pick_bn(int N) {
  // minimise padded columns; ties go to the wider tile (fewer A re-reads)
  int best = 128, best_pad = cdiv(N, 128) * 128;
  for (int bn : {64, 32}) {
    int pad = cdiv(N, bn) * bn;
    if (pad < best_pad) { best = bn; best_pad = pad; }
  }
  return best;
}

template <typename T, bool BT, bool LAZY>
static int dispatch_gemm(GemmArgs g, hipStream_t s) {
  const int bn = pick_bn(g.N);
  const bool big = (long)cdiv(g.M, 128) * cdiv(g.N, bn) >= 512;
  if (big) {
    if (bn == 128) return launch_gemm<T, 128, 128, BT, LAZY>(g, s);
    if (bn == 64) return launch_gemm<T, 128, 64, BT, LAZY>(g, s);
    return launch_gemm<T, 128, 32, BT, LAZY>(g, s);
  }
  if (bn == 128) return launch_gemm<T, 64, 128, BT, LAZY>(g, s);
  if (bn == 64) return launch_gemm<T, 64, 64, BT, LAZY>(g, s);
  return launch_gemm<T, 64, 32, BT, LAZY>(g, s);
}

static bool lazy_is_plain(const edet_lazy* a) {
  return a->bn.enabled == 0 && a->act == EDET_ACT_NONE && a->gate == nullptr;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_conv1x1_fwd(int dtype, const edet_lazy* a, const edet_pyramid* rows, int K,
                     const void* wt, int N, const float* bias, void* y, int ldy,
                     int accumulate, const edet_segout* stats, edet_stream_t stream) {
  EDET_REQUIRE(a && rows && wt && y, "conv1x1_fwd: null argument");
  EDET_REQUIRE(K > 0 && N > 0 && a->ld % 8 == 0 && K % 8 == 0 && K <= 8192,
               "conv1x1_fwd: need K%%8==0, lda%%8==0 (K=%d lda=%d)", K, a->ld);
  EDET_REQUIRE(rows->nseg >= 1 && rows->nseg <= EDET_MAX_SEG, "conv1x1_fwd: bad pyramid");
  EDET_REQUIRE(a->gate == nullptr || rows->nseg == 1, "conv1x1_fwd: gate needs 1 segment");
  GemmArgs g{};
  g.a = a->x; g.b = wt; g.c = y; g.bias = bias; g.lz = *a; g.pyr = *rows;
  g.lda = a->ld; g.ldb = K; g.ldc = ldy; g.M = pyr_total_rows(*rows); g.K = K; g.N = N;
  g.accumulate = accumulate;
  g.has_stats = stats != nullptr;
  if (stats) g.stats = *stats;
  hipStream_t s = (hipStream_t)stream;
  const bool plain = lazy_is_plain(a);
  EDET_DTYPE_DISPATCH(dtype, T, {
    return plain ? dispatch_gemm<T, true, false>(g, s) : dispatch_gemm<T, true, true>(g, s);
  });
}

int edet_conv1x1_dgrad(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                       const void* wt, int K, void* dx, int lddx, int accumulate,
                       edet_stream_t stream) {
  EDET_REQUIRE(dy && rows && wt && dx, "conv1x1_dgrad: null argument");
  EDET_REQUIRE(lddy % 8 == 0 && K % 8 == 0 && N > 0, "conv1x1_dgrad: need lddy%%8==0, K%%8==0");
  GemmArgs g{};
  g.a = dy; g.b = wt; g.c = dx; g.bias = nullptr; g.pyr = *rows;
  g.lda = lddy; g.ldb = K; g.ldc = lddx;
  g.M = pyr_total_rows(*rows); g.K = N; g.N = K;  // GEMM K = conv out channels
  g.accumulate = accumulate; g.has_stats = 0;
  hipStream_t s = (hipStream_t)stream;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_gemm<T, false, false>(g, s); });
}

int edet_conv1x1_wgrad(int dtype, const edet_lazy* a, const edet_pyramid* rows, int K,
                       const void* dy, int lddy, int N, float* dwt, float* dbias,
                       edet_stream_t stream) {
  EDET_REQUIRE(a && rows && dy && dwt, "conv1x1_wgrad: null argument");
  EDET_REQUIRE(a->ld % 8 == 0 && lddy % 8 == 0 && K > 0 && N > 0,
               "conv1x1_wgrad: need lda%%8==0, lddy%%8==0");
  EDET_REQUIRE(a->gate == nullptr || rows->nseg == 1, "conv1x1_wgrad: gate needs 1 segment");
  WgradArgs g{};
  g.a = a->x; g.dy = dy; g.dw = dwt; g.db = dbias; g.lz = *a; g.pyr = *rows;
  g.lda = a->ld; g.lddy = lddy; g.M = pyr_total_rows(*rows); g.K = K; g.N = N;
  g.ntn = cdiv(N, 64); g.ntk = cdiv(K, 64);
  const int tiles = g.ntn * g.ntk;
  int split = cdiv(2048, tiles);
  const int max_split = cdiv(g.M, 32 * 4);  // at least 4 row-chunks per block
  if (split > max_split) split = max_split;
  if (split < 1) split = 1;
  g.rows_per = cdiv(cdiv(g.M, split), 32) * 32;
  split = cdiv(g.M, g.rows_per);
  if (split < 1) split = 1;
  hipStream_t s = (hipStream_t)stream;
  const bool plain = lazy_is_plain(a);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (plain) hipLaunchKernelGGL((k_wgrad<T, false>), dim3(tiles * split), dim3(256), 0, s, g);
    else hipLaunchKernelGGL((k_wgrad<T, true>), dim3(tiles * split), dim3(256), 0, s, g);
    return check_launch("edet wgrad");
  });
}

}  // extern "C"
