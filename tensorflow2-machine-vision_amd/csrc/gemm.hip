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
#include <type_traits>

#include "common.hpp"

namespace edet {


struct GemmArgs {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  edet_lazy lz;
  edet_pyramid pyr;
  edet_statout stats;  // BN statistics of y, or (FOLD) the folded sums: sum <- dbeta, sq <- dgamma
  edet_lazy fx;        // FOLD: the value whose gradient y is (raw x, BN, act; no gate)
  int lda, ldb, ldc, M, K, N;
  int accumulate, has_stats, ntm, ntn;
  double* se5;         // FOLD == 2: [5][se_batch][N] per-image SE / BN-backward sums (k_gate_bn_reduce's)
  int se_batch;
  int ncs;             // k_gemm_s: column slices of 16 NF columns (0 / 1: one, the whole N)
};

// BN-backward fold (dgrad epilogues): the output y = d(value) of a lazy value v = act(bn(x)) is
// turned into the two per-channel sums edet_lazy_bwd_reduce would take in its own pass,
//   du = y * act'(bn(x)),  dbeta += du,  dgamma += du * xhat,
// from the stored (storage-rounded) y, so the apply pass that later reads y uses sums of exactly
// the values it applies them to.  Per channel: (bn scale, bn shift, mean, rstd).
__device__ __forceinline__ float4 fold_table(const edet_bn& bn, int seg, int c, float inv_count) {
  const float2 af = bn_affine(bn, seg, c, inv_count), mr = bn_mean_rstd(bn, seg, c, inv_count);
  return make_float4(af.x, af.y, mr.x, mr.y);
}
__device__ __forceinline__ void fold_terms(float y, float x, const float4& t, int act, float& du, float& dux) {
  du = act ? y * dswishf_(x * t.x + t.y) : y;
  dux = du * ((x - t.z) * t.w);
}

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

// Rows [0, nrows) of a row-major [.][ld] matrix, columns [0, KP) (KP % 8 == 0), into LDS
// [nrows][lds_ld] with 8 16-byte vectors per thread in flight before any is stored (cp8 per
// vector waits for each load inside its branch: one round trip per vector, 7 per 64-row chunk at
// K = 224); rows at or past nvalid and elements at or past K are written as zeros.
template <typename T>
__device__ __forceinline__ void stage_rows(T* lds, int lds_ld, const T* src, int ld, int nrows, int nvalid,
                                           int K, int KP) {
  using V = typename std::conditional<sizeof(T) == 2, uint4, float4>::type;
  constexpr int VW = sizeof(T) == 2 ? 1 : 2, U = 8;
  const int kv8 = KP / 8, total = nrows * kv8;
  // range-checked loads: rows at or past nvalid read zeros, vectors at or past K take an
  // out-of-range offset (a select on each loaded value made the compiler wait for it at once)
  const auto rs = buf_rsrc(src, (long)min(nrows, nvalid) * ld * (long)sizeof(T));
  for (int v0 = 0; v0 < total; v0 += 256 * U) {
    V t[U][VW];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = v0 + threadIdx.x + u * 256;
      const int n = v / kv8, kv = (v - n * kv8) * 8;
      const uint32_t off = buf_off(v < total && kv < K, (uint32_t)((n * ld + kv) * (int)sizeof(T)));
#pragma unroll
      for (int w = 0; w < VW; ++w) t[u][w] = __builtin_bit_cast(V, buf_ld16(rs, off + 16 * w));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = v0 + threadIdx.x + u * 256;
      const int n = v / kv8, kv = (v - n * kv8) * 8;
      if (v < total && kv < K && K - kv < 8) {  // tail vector: zero the elements at or past K
        T* e = reinterpret_cast<T*>(&t[u][0]);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j >= K - kv) e[j] = T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = v0 + threadIdx.x + u * 256;
      if (v < total) {
        const int n = v / kv8, kv = (v - n * kv8) * 8;
#pragma unroll
        for (int w = 0; w < VW; ++w) reinterpret_cast<V*>(lds + (size_t)n * lds_ld + kv)[w] = t[u][w];
      }
    }
  }
}

__device__ __forceinline__ bf16x8_t lds_frag_bf16(const uint16_t* p) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  return __builtin_bit_cast(bf16x8_t, v);
}

// images a BM-row tile of one segment can span (the staged SE gate rows of k_gemm)
__host__ __device__ __forceinline__ int gemm_gate_imgs(int BM, int hw, int batch) {
  return min(batch, (BM - 1) / hw + 2);
}

// K-streaming GEMM for K > 512 (the MBConv project convs, K = 480 ... 1152, N <= 320): one
// block owns a BM x BN tile with the whole N, and walks K in 32-wide chunks.  Software
// pipelined: chunk k+1 is fetched global -> registers while chunk k's MFMAs run, LDS is
// double-buffered, one barrier per chunk (the unpipelined loop exposed the full load latency
// 36 times per tile: 150 GB/s at M = 8192).  B is the [N][K] weight (k contiguous).
// FOLD == 1: the BN-backward fold above.  FOLD == 2 (edet_conv1x1_dgrad_sesum, the MBConv
// project conv's dgrad): y = d(value) of the SE-gated v = swish(bn(x)) * gate, and the epilogue
// takes k_gate_bn_reduce's five per-image sums from the stored y and the x tile (a tile lies in
// one image: the host requires H*W % BM == 0), flushed as fp64 atomics per (sum, image, column)
// ACC (accumulating dgrads, compile-time: the model's multi-consumer gradients): the C tile is
// staged in fp32 and the store adds it to the old value, one rounding to the storage type (a
// staged round(v) added later rounded twice; a runtime accumulate test in the staging loop cost
// 2-9 us on every K-loop launch, r05c)
template <typename T, int BM, int BN, int KC, bool LAZY, int FOLD = 0, bool ACC = false>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  constexpr int KV = KC / 8, LDK = KC + 8;
  constexpr int AV = (BM * KV + 255) / 256, BV = (BN * KV + 255) / 256;
  using V = typename std::conditional<sizeof(T) == 2, uint4, float4>::type;
  constexpr int VW = sizeof(T) == 2 ? 1 : 2;  // 16-byte words per 8 elements
  // A / B chunk buffers, reused after the K loop as the C tile staged for 16-byte row stores
  // (FOLD: and the folded value's raw x tile behind it)
  constexpr int LDC_S = BN + 8;
  constexpr int AB_BYTES = 2 * (BM + BN) * LDK * (int)sizeof(T);
  constexpr int C_BYTES = (FOLD ? 2 : 1) * BM * LDC_S * (int)(ACC ? sizeof(float) : sizeof(T));
  __shared__ __attribute__((aligned(16))) char smem_ab[AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES];
  T (*As)[BM * LDK] = reinterpret_cast<T (*)[BM * LDK]>(smem_ab);
  T (*Bs)[BN * LDK] = reinterpret_cast<T (*)[BN * LDK]>(smem_ab + 2 * BM * LDK * sizeof(T));
  T* Cs = reinterpret_cast<T*>(smem_ab);
  float* Cf = reinterpret_cast<float*>(smem_ab);  // ACC: the fp32 C tile
  T* Xs = Cs + BM * LDC_S;         // FOLD
  __shared__ float4 ftab[FOLD ? BN : 1];
  __shared__ float red[FOLD == 2 ? 5 : 2][2][BN];  // [sum|sq (5 SE sums)][wm][col]: one writer each
  extern __shared__ float2 xf[];   // [K] lazy affine per input channel, then [images][K] gate rows
  float* gts = reinterpret_cast<float*>(xf + (LAZY ? g.K : 0));

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = t / g.ntn, tn = t - tm * g.ntn;
  const int row0 = tm * BM, col0 = tn * BN;

  const T* A = (const T*)g.a;
  const T* B = (const T*)g.b;
  struct Chunk {
    V ra[AV][VW], rb[BV][VW];
  };
  // global -> registers (raw), branch-free: an element outside the operand reads zeros
  // (buf_ld16).  Loads under branches left the compiler's wait-count merge pessimistic: every
  // commit waited for the chunks in flight behind it (s_waitcnt vmcnt(0)).
  // (range-checked loads over the block's A rows / B rows: rows past M or N read zeros, a
  // chunk column past K takes an out-of-range offset)
  const auto ra_ = buf_rsrc(A + (size_t)row0 * g.lda, (long)min(BM, g.M - row0) * g.lda * (long)sizeof(T));
  const auto rb_ = buf_rsrc(B + (size_t)col0 * g.ldb, (long)min(BN, g.N - col0) * g.ldb * (long)sizeof(T));
  auto fetch = [&](Chunk& R, int k0) {
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int v = tid + u * 256;
      const int r = v / KV, kv = (v % KV) * 8;
      const uint32_t off = buf_off(v < BM * KV && k0 + kv < g.K, (uint32_t)((r * g.lda + k0 + kv) * (int)sizeof(T)));
#pragma unroll
      for (int w = 0; w < VW; ++w) R.ra[u][w] = __builtin_bit_cast(V, buf_ld16(ra_, off + 16 * w));
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      const int v = tid + u * 256;
      const int n = v / KV, kv = (v % KV) * 8;
      const uint32_t off = buf_off(v < BN * KV && k0 + kv < g.K, (uint32_t)((n * g.ldb + k0 + kv) * (int)sizeof(T)));
#pragma unroll
      for (int w = 0; w < VW; ++w) R.rb[u][w] = __builtin_bit_cast(V, buf_ld16(rb_, off + 16 * w));
    }
  };
  // chunk 0 is requested before the per-block tables (lazy affine, gate rows, fold table) are
  // built: its round trip overlaps theirs instead of following the barrier
  Chunk R0, R1;
  fetch(R0, 0);

  int seg = 0;
  if (LAZY || g.has_stats) seg = seg_of_row(g.pyr, row0);
  const int seg_off = g.pyr.row_off[seg];
  const int seg_end = seg_off + seg_rows(g.pyr, seg);
  const int hw = g.pyr.H[seg] * g.pyr.W[seg];
  if constexpr (FOLD) {
    const float inv = 1.f / (float)seg_rows(g.pyr, seg);
    for (int c = tid; c < BN; c += 256)
      ftab[c] = col0 + c < g.N ? fold_table(g.fx.bn, seg, col0 + c, inv) : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // SE gate rows of the images this tile spans (gemm_gate_imgs of them), staged in LDS once:
  // per-element global gate loads sat on the chunk loop's critical path
  const bool has_gate = LAZY && g.lz.gate != nullptr;
  const int n_lo = (row0 - seg_off) / hw;
  if constexpr (LAZY) {
    const float inv = 1.f / (float)seg_rows(g.pyr, seg);
    for (int k = tid; k < g.K; k += 256) xf[k] = bn_affine(g.lz.bn, seg, k, inv);
    if (has_gate) {
      const int ni = gemm_gate_imgs(BM, hw, g.pyr.batch);
      for (int e = tid; e < ni * g.K; e += 256) {
        const int i = e / g.K, k = e - i * g.K, n = n_lo + i;
        gts[e] = (n < g.pyr.batch) ? g.lz.gate[(size_t)n * g.K + k] : 0.f;
      }
    }
  }
  __syncthreads();

  // FOLD: the folded value's x tile is requested here, its latency hidden by the whole K loop,
  // and parked in LDS next to the staged C tile after it
  constexpr int VPR = BN / 8;  // 8-element vectors per tile row
  constexpr int NXV = FOLD ? (BM * VPR + 255) / 256 : 1;
  V xr[NXV][VW];
  if constexpr (FOLD) {
    const T* X = (const T*)g.fx.x;
#pragma unroll
    for (int u = 0; u < NXV; ++u) {
      const int e = tid + u * 256, rl = e / VPR, cv = (e - rl * VPR) * 8;
      const int row = row0 + rl, col = col0 + cv;
      const bool ok = e < BM * VPR && row < g.M && col < g.N;  // N % 8 == 0: whole vectors
      const V* src = reinterpret_cast<const V*>(X + (ok ? (size_t)row * g.fx.ld + col : 0));
#pragma unroll
      for (int w = 0; w < VW; ++w) xr[u][w] = ok ? src[w] : V{};
    }
  }
  // per-thread A rows are fixed across chunks: resolve their staged gate rows once
  int goff[AV];
#pragma unroll
  for (int u = 0; u < AV; ++u) {
    const int grow = min(row0 + (tid + u * 256) / KV, g.M - 1);
    goff[u] = has_gate ? ((grow - seg_off) / hw - n_lo) * g.K : 0;
  }
  // registers -> LDS buffer, lazy transform of A on the way: branch-free per element (the
  // activation and the gate are block-uniform choices, taken once around the whole chunk)
  auto lazy_a = [&](auto act_c, auto gate_c, const Chunk& R, int buf, int k0) {
    constexpr bool ACT = decltype(act_c)::value, GATE = decltype(gate_c)::value;
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int v = tid + u * 256;
      if (v < BM * KV) {
        const int r = v / KV, kv = (v % KV) * 8, gk = k0 + kv;
        const bool rok = row0 + r < g.M;
        const T* e = reinterpret_cast<const T*>(&R.ra[u][0]);
        float vals[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = min(gk + j, g.K - 1);
          float x = to_f<T>(e[j]) * xf[k].x + xf[k].y;
          if constexpr (ACT) x = swishf_(x);
          if constexpr (GATE) x *= gts[goff[u] + k];
          vals[j] = (rok && gk + j < g.K) ? x : 0.f;
        }
        st8(&As[buf][r * LDK + kv], vals);
      }
    }
  };
  auto commit = [&](const Chunk& R, int buf, int k0) {
    if constexpr (LAZY) {
      using TT = std::true_type;
      using FF = std::false_type;
      if (g.lz.act) {
        if (has_gate) lazy_a(TT{}, TT{}, R, buf, k0);
        else lazy_a(TT{}, FF{}, R, buf, k0);
      } else {
        if (has_gate) lazy_a(FF{}, TT{}, R, buf, k0);
        else lazy_a(FF{}, FF{}, R, buf, k0);
      }
    }
#pragma unroll
    for (int u = 0; u < AV; ++u) {
      const int v = tid + u * 256;
      if (v < BM * KV) {
        const int r = v / KV, kv = (v % KV) * 8;
        T* dst = &As[buf][r * LDK + kv];
        if constexpr (!LAZY) {
#pragma unroll
          for (int w = 0; w < VW; ++w) reinterpret_cast<V*>(dst)[w] = R.ra[u][w];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < BV; ++u) {
      const int v = tid + u * 256;
      if (v < BN * KV) {
        const int n = v / KV, kv = (v % KV) * 8;
#pragma unroll
        for (int w = 0; w < VW; ++w) reinterpret_cast<V*>(&Bs[buf][n * LDK + kv])[w] = R.rb[u][w];
      }
    }
  };

  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Two register chunks in flight: chunk k+1 was fetched two iterations before its commit (one
  // chunk ahead left every 32-wide K step waiting a memory round trip behind a handful of MFMAs)
  const int nk = cdiv(g.K, KC);
  commit(R0, 0, 0);
  fetch(R0, KC);  // (past K: every element is outside, committed as zeros or not at all)
  fetch(R1, 2 * KC);
  __syncthreads();
  auto kstep = [&](Chunk& R, int kt) {
    const int buf = kt & 1;
    const T* Ab = As[buf];
    const T* Bb = Bs[buf];
#pragma unroll
    for (int ks = 0; ks < KC; ks += 32) {
      if constexpr (sizeof(T) == 2) {
        bf16x8_t af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = lds_frag_bf16(&Ab[(wm * WM + i * 16 + (lane & 15)) * LDK + ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = lds_frag_bf16(&Bb[(wn * WN + j * 16 + (lane & 15)) * LDK + ks + 8 * (lane >> 4)]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          float af[FM], bfr[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) af[i] = Ab[(wm * WM + i * 16 + (lane & 15)) * LDK + ks + 4 * s + (lane >> 4)];
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[j] = Bb[(wn * WN + j * 16 + (lane & 15)) * LDK + ks + 4 * s + (lane >> 4)];
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    commit(R, buf ^ 1, (kt + 1) * KC);
    fetch(R, (kt + 3) * KC);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    kstep(R0, kt);
    if (kt + 1 < nk) kstep(R1, kt + 1);
  }

  // ---- epilogue: bias, BN statistics, the tile staged in LDS (the K loop's last barrier freed
  // the chunk buffers), then written as 16-byte row vectors (the MFMA layout's per-lane 2-byte
  // stores left 32-byte pieces of lines: 8192 x 192 -> 1152 ran at 0.65 TB/s)
  T* C = (T*)g.c;
  float ssum[FN], ssq[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) { ssum[j] = 0.f; ssq[j] = 0.f; }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int cl = wn * WN + j * 16 + (lane & 15), col = col0 + cl;
    const float bv = (g.bias && col < g.N) ? g.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rl = wm * WM + i * 16 + (lane >> 4) * 4 + r, row = row0 + rl;
        const float v = acc[i][j][r] + bv;
        if constexpr (ACC) Cf[rl * LDC_S + cl] = v;
        else Cs[rl * LDC_S + cl] = from_f<T>(v);
        if (FOLD == 0 && row < g.M && col < g.N && row < seg_end) { ssum[j] += v; ssq[j] += v * v; }
      }
    }
  }
  if constexpr (FOLD) {
#pragma unroll
    for (int u = 0; u < NXV; ++u) {
      const int e = tid + u * 256, rl = e / VPR, cv = (e - rl * VPR) * 8;
      if (e < BM * VPR) {
#pragma unroll
        for (int w = 0; w < VW; ++w) reinterpret_cast<V*>(Xs + rl * LDC_S + cv)[w] = xr[u][w];
      }
    }
  }
  __syncthreads();
  float se[FOLD == 2 ? 5 : 1][FOLD == 2 ? FN : 1];
  if constexpr (FOLD == 2) {  // k_gate_bn_reduce's terms of the stored (rounded) y, same formulas
#pragma unroll
    for (int q = 0; q < 5; ++q)
#pragma unroll
      for (int j = 0; j < FN; ++j) se[q][j] = 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cl = wn * WN + j * 16 + (lane & 15), col = col0 + cl;
      const float4 t = ftab[cl];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = wm * WM + i * 16 + (lane >> 4) * 4 + r, row = row0 + rl;
          const float k = (row < g.M && col < g.N && row < seg_end) ? 1.f : 0.f;
          const float xv = to_f<T>(Xs[rl * LDC_S + cl]);
          const float uu = xv * t.x + t.y;
          const float sg = sigmoidf_(uu);
          const float sw = uu * sg, dsw = sg * (1.f + uu * (1.f - sg)) * k;
          const float xh = (xv - t.z) * t.w;
          const float dd = to_f<T>(Cs[rl * LDC_S + cl]) * k;
          se[0][j] += dd * sw;
          se[1][j] += dd * dsw;
          se[2][j] += dsw;
          se[3][j] += dd * dsw * xh;
          se[4][j] += dsw * xh;
        }
      }
    }
  } else if constexpr (FOLD == 1) {  // sums of the stored (rounded) values, in the statistics' layout
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cl = wn * WN + j * 16 + (lane & 15), col = col0 + cl;
      const float4 t = ftab[cl];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = wm * WM + i * 16 + (lane >> 4) * 4 + r, row = row0 + rl;
          if (row < g.M && col < g.N && row < seg_end) {
            float du, dux;
            fold_terms(to_f<T>(Cs[rl * LDC_S + cl]), to_f<T>(Xs[rl * LDC_S + cl]), t, g.fx.act, du, dux);
            ssum[j] += du;
            ssq[j] += dux;
          }
        }
      }
    }
  }
  {
    for (int e = tid; e < BM * VPR; e += 256) {
      const int rl = e / VPR, cv = (e - rl * VPR) * 8;
      const int row = row0 + rl, col = col0 + cv;
      if (row < g.M && col < g.N) {
        float vals[8];
        const T* src = Cs + rl * LDC_S + cv;
        if constexpr (ACC) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) vals[jj] = Cf[rl * LDC_S + cv + jj];
        } else {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) vals[jj] = to_f<T>(src[jj]);
        }
        acc8m(C + (size_t)row * g.ldc + col, g.N - col, vals, ACC ? 1 : 0);
      }
    }
  }
  if constexpr (FOLD == 2) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const float v = row4_sum(se[q][j]);
        if (lane < 16) red[q][wm][wn * WN + j * 16 + lane] = v;
      }
    __syncthreads();
    const int n = (row0 - seg_off) / hw;
    for (int e = tid; e < 5 * BN; e += 256) {
      const int q = e / BN, i = e - q * BN, col = col0 + i;
      if (col < g.N && row0 < g.M)
        stat_add(g.se5 + ((size_t)q * g.se_batch + n) * g.N + col, (double)(red[q][0][i] + red[q][1][i]));
    }
    return;
  }
  if (g.has_stats) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      float s = ssum[j], q = ssq[j];
      s = row4_sum(s);
      q = row4_sum(q);
      if (lane < 16) {
        red[0][wm][wn * WN + j * 16 + lane] = s;
        red[1][wm][wn * WN + j * 16 + lane] = q;
      }
    }
    __syncthreads();
    for (int i = tid; i < BN; i += 256) {
      const int col = col0 + i;
      if (col < g.N) {
        stat_put(g.stats.sum[seg], col, (double)(red[0][0][i] + red[0][1][i]));
        stat_put(g.stats.sq[seg], col, (double)(red[1][0][i] + red[1][1][i]));
      }
    }
  }
}

// ------------------------------------------------------------------ A-resident GEMM
// One workgroup owns BM rows and keeps its whole (lazily transformed) A tile [BM][K] in LDS,
// then walks its columns in 64-wide chunks (A is read from HBM exactly once whatever N is —
// the expand convs have N = 6K).  The whole C tile [BM][cols] is staged in LDS and written
// back as one linear stream of 16-byte stores (rows are contiguous when ldc == N), so HBM
// sees full cache lines.  For small M the columns are split over `nsplit` workgroups per row
// tile (A re-read from L2) so the grid still fills the 256 CUs.
constexpr int RNB = 64;

template <typename T, int BM, bool LAZY>
__global__ __launch_bounds__(256) void k_gemm_r(GemmArgs g, int KP, int nsplit, int cps, int LDC, int bstage) {
  constexpr int WM = BM / 2, FM = WM / 16, FN = 2;
  const int LDA = KP + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // B chunks are double-buffered and fetched one chunk ahead when a chunk is at most 4
  // vectors per thread (KP <= 128); wider K keeps one buffer and loads each chunk in place
  const bool bpipe = KP <= 128;
  T* As = reinterpret_cast<T*>(smem);
  T* Bs = As + BM * LDA;                                  // [bpipe ? 2 : 1][RNB][LDA]
  T* Cs = Bs + (bpipe ? 2 : 1) * RNB * LDA;               // [BM][LDC] (this split's columns)
  // per-block BN partials [sum|sq][wm][LDC]: each entry has exactly one writer lane, and the
  // two wm halves are added in a fixed order at the flush (LDS float atomics would make the
  // block partial depend on wave timing, and BN statistics must be reproducible)
  float* red = reinterpret_cast<float*>(Cs + BM * LDC);
  float* bias_s = red + 4 * LDC;                           // [LDC] this split's bias
  float2* xf = reinterpret_cast<float2*>(bias_s + LDC);    // [K] (LAZY)
  float* gt = reinterpret_cast<float*>(xf + (LAZY ? g.K : 0));  // [images][K] SE gate rows (LAZY)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // persistent: block w owns column split (w % nsplit) and every G-th row tile, so the BN
  // statistics leave the block once per segment instead of once per tile (same-address
  // atomics from thousands of tiles serialise in L2).
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int G = gridDim.x / nsplit;
  const int split = w % nsplit, wt = w / nsplit;
  const int K = g.K, N = g.N;
  const int ntm = cdiv(g.M, BM);
  const int ch_begin = split * cps;
  const int ch_end = min(cdiv(N, RNB), ch_begin + cps);
  if (ch_begin >= ch_end) return;
  const int cbase = ch_begin * RNB;                      // first column of this split
  const int ncols = min(N, ch_end * RNB) - cbase;         // valid columns of this split
  for (int c = tid; c < 4 * LDC; c += 256) red[c] = 0.f;
  for (int c = tid; c < LDC; c += 256) bias_s[c] = (g.bias && c < ncols) ? g.bias[cbase + c] : 0.f;
  int cur_seg = -1;

  // A tile rows: vector v = v0 + tid + u*256 is row v / kv8, channels (v % kv8) * 8 .. +8
  const T* A = (const T*)g.a;
  const int kv8 = KP / 8;
  using V = typename std::conditional<sizeof(T) == 2, uint4, float4>::type;
  constexpr int VW = sizeof(T) == 2 ? 1 : 2, UNR = 4;
  // range-checked loads (rows past M, columns past K read zeros): every load is issued
  // unconditionally and needs no select, so the compiler does not wait for it where it is issued
  auto fetch_a = [&](V (&raw)[UNR][VW], int tmt, int v0) {
    const auto rs = buf_rsrc(A + (size_t)tmt * BM * g.lda, (long)min(BM, g.M - tmt * BM) * g.lda * (long)sizeof(T));
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int v = v0 + tid + u * 256;
      const int r = v / kv8, kv = (v - r * kv8) * 8;
      const uint32_t off = buf_off(v < BM * kv8 && kv < K, (uint32_t)((r * g.lda + kv) * (int)sizeof(T)));
#pragma unroll
      for (int w = 0; w < VW; ++w) raw[u][w] = __builtin_bit_cast(V, buf_ld16(rs, off + 16 * w));
    }
  };
  const bool has_gate = LAZY && g.lz.gate != nullptr;
  auto lazy_a = [&](auto act_c, auto gate_c, const V (&raw)[UNR][VW], int v0, int row0, int seg_off, int hw, int n_lo) {
    constexpr bool ACT = decltype(act_c)::value, GATE = decltype(gate_c)::value;
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int v = v0 + tid + u * 256;
      if (v >= BM * kv8) break;
      const int r = v / kv8, kv = (v - r * kv8) * 8;
      const int grow = row0 + r;
      const bool live = grow < g.M && kv < K;
      const int gbase = GATE ? ((min(grow, g.M - 1) - seg_off) / hw - n_lo) * K : 0;
      const T* e = reinterpret_cast<const T*>(&raw[u][0]);
      float vals[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = min(kv + j, K - 1);
        float x = to_f<T>(e[j]) * xf[k].x + xf[k].y;
        if constexpr (ACT) x = swishf_(x);
        if constexpr (GATE) x *= gt[gbase + k];
        vals[j] = live ? x : 0.f;
      }
      st8(&As[r * LDA + kv], vals);
    }
  };
  auto commit_a = [&](const V (&raw)[UNR][VW], int v0, int row0, int seg_off, int hw, int n_lo) {
    if constexpr (LAZY) {
      using TT = std::true_type;
      using FF = std::false_type;
      if (g.lz.act) {
        if (has_gate) lazy_a(TT{}, TT{}, raw, v0, row0, seg_off, hw, n_lo);
        else lazy_a(TT{}, FF{}, raw, v0, row0, seg_off, hw, n_lo);
      } else {
        if (has_gate) lazy_a(FF{}, TT{}, raw, v0, row0, seg_off, hw, n_lo);
        else lazy_a(FF{}, FF{}, raw, v0, row0, seg_off, hw, n_lo);
      }
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int v = v0 + tid + u * 256;
        if (v >= BM * kv8) break;
        const int r = v / kv8, kv = (v - r * kv8) * 8;
#pragma unroll
        for (int w = 0; w < VW; ++w) reinterpret_cast<V*>(&As[r * LDA + kv])[w] = raw[u][w];
      }
    }
  };
  const bool apre = BM * kv8 <= 256 * UNR;
  V araw[UNR][VW];
  if (apre && wt < ntm) fetch_a(araw, wt, 0);
  const bool bres = ch_end - ch_begin == 1;  // this split's B chunk stays in LDS for every tile
  const T* B = (const T*)g.b;
  using VB = typename std::conditional<sizeof(T) == 2, uint4, float4>::type;
  constexpr int VWB = sizeof(T) == 2 ? 1 : 2, NBV = 4;
  VB rb[NBV][VWB];
  auto load_b = [&](int ch, T* bs) {  // in place (global -> LDS)
    if (bstage) {
      stage_rows(bs, LDA, B + (size_t)ch * RNB * g.ldb, g.ldb, RNB, N - ch * RNB, K, KP);
      return;
    }
    for (int v = tid; v < RNB * kv8; v += 256) {
      const int n = v / kv8, kv = (v - n * kv8) * 8;
      const int gn = ch * RNB + n, nk = K - kv;
      T* dst = &bs[n * LDA + kv];
      if (gn < N && nk > 0) cp8(dst, B + (size_t)gn * g.ldb + kv, nk);
      else zero8(dst);
    }
  };
  auto fetch_b = [&](int ch) {  // registers, range-checked (K % 8 == 0)
    const auto rs = buf_rsrc(B + (size_t)ch * RNB * g.ldb, (long)min(RNB, N - ch * RNB) * g.ldb * (long)sizeof(T));
#pragma unroll
    for (int u = 0; u < NBV; ++u) {
      const int v = tid + u * 256;
      const int n = v / kv8, kv = (v - n * kv8) * 8;
      const uint32_t off = buf_off(v < RNB * kv8 && kv < K, (uint32_t)((n * g.ldb + kv) * (int)sizeof(T)));
#pragma unroll
      for (int w = 0; w < VWB; ++w) rb[u][w] = __builtin_bit_cast(VB, buf_ld16(rs, off + 16 * w));
    }
  };
  auto commit_b = [&](T* bs) {
#pragma unroll
    for (int u = 0; u < NBV; ++u) {
      const int v = tid + u * 256;
      if (v >= RNB * kv8) break;
      const int n = v / kv8, kv = (v - n * kv8) * 8;
#pragma unroll
      for (int w = 0; w < VWB; ++w) reinterpret_cast<VB*>(&bs[n * LDA + kv])[w] = rb[u][w];
    }
  };
  if (bres) load_b(ch_begin, Bs);  // (visible after the first tile's barrier)

  for (int tm = wt; tm < ntm; tm += G) {
  const int row0 = tm * BM;
  const int seg = seg_of_row(g.pyr, row0);
  const int seg_off = g.pyr.row_off[seg];
  const int seg_end = seg_off + seg_rows(g.pyr, seg);
  const int hw = g.pyr.H[seg] * g.pyr.W[seg];
  if (seg != cur_seg) {
    __syncthreads();
    if (cur_seg >= 0 && g.has_stats)
      for (int c = tid; c < ncols; c += 256) {
        stat_put(g.stats.sum[cur_seg], cbase + c, (double)(red[c] + red[LDC + c]));
        stat_put(g.stats.sq[cur_seg], cbase + c, (double)(red[2 * LDC + c] + red[3 * LDC + c]));
        red[c] = red[LDC + c] = red[2 * LDC + c] = red[3 * LDC + c] = 0.f;
      }
    if constexpr (LAZY) {
      const float inv = 1.f / (float)seg_rows(g.pyr, seg);
      for (int k = tid; k < K; k += 256) xf[k] = bn_affine(g.lz.bn, seg, k, inv);
    }
    cur_seg = seg;
    __syncthreads();
  }
  // ---- SE gate rows of this tile's images in LDS (gemm_gate_imgs of them)
  const int n_lo = (row0 - seg_off) / hw;
  if (has_gate) {
    const int ni = gemm_gate_imgs(BM, hw, g.pyr.batch);
    for (int e = tid; e < ni * K; e += 256) {
      const int i = e / K, k = e - i * K, n = n_lo + i;
      gt[e] = (n < g.pyr.batch) ? g.lz.gate[(size_t)n * K + k] : 0.f;
    }
    __syncthreads();
  }
  // ---- A tile (once per row tile); UNR vector loads in flight per thread before any use.
  // When the whole tile is one round of UNR vectors per thread, the next tile's round is
  // fetched here and committed at the next tile's start (its HBM latency overlaps this tile's
  // MFMAs, epilogue and write-out)
  if (apre) {
    commit_a(araw, 0, row0, seg_off, hw, n_lo);
  } else {
    for (int v0 = 0; v0 < BM * kv8; v0 += 256 * UNR) {
      V raw[UNR][VW];
      fetch_a(raw, tm, v0);
      commit_a(raw, v0, row0, seg_off, hw, n_lo);
    }
  }
  if (!bres) load_b(ch_begin, Bs);
  // (after the in-place B loads: their waits would drain it -- the wait counter is in order)
  if (apre && tm + G < ntm) fetch_a(araw, tm + G, 0);
  __syncthreads();
  if (bpipe && ch_begin + 1 < ch_end) fetch_b(ch_begin + 1);
  for (int ch = ch_begin; ch < ch_end; ++ch) {
    const int col0 = ch * RNB;
    T* Bc = Bs + (bpipe ? ((ch - ch_begin) & 1) * RNB * LDA : 0);
    if (!bpipe && ch > ch_begin) {
      load_b(ch, Bs);
      __syncthreads();
    }

    floatx4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < KP; k0 += 32) {
      if constexpr (sizeof(T) == 2) {
        bf16x8_t af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = lds_frag_bf16(&As[(wm * WM + i * 16 + (lane & 15)) * LDA + k0 + 8 * (lane >> 4)]);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = lds_frag_bf16(&Bc[(wn * 32 + j * 16 + (lane & 15)) * LDA + k0 + 8 * (lane >> 4)]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          float af[FM], bfr[FN];
#pragma unroll
          for (int i = 0; i < FM; ++i) af[i] = As[(wm * WM + i * 16 + (lane & 15)) * LDA + k0 + 4 * s + (lane >> 4)];
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[j] = Bc[(wn * 32 + j * 16 + (lane & 15)) * LDA + k0 + 4 * s + (lane >> 4)];
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    // bias, BN statistics (fp32, accumulated in LDS across tiles), stage into the C tile
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cl = wn * 32 + j * 16 + (lane & 15);
      const int col = col0 + cl;
      const float bv = col - cbase < LDC ? bias_s[col - cbase] : 0.f;
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = wm * WM + i * 16 + (lane >> 4) * 4 + r;
          const float v = acc[i][j][r] + bv;
          if (col - cbase < LDC) Cs[rl * LDC + col - cbase] = from_f<T>(v);
          if (row0 + rl < seg_end && col < N) { s += v; q += v * v; }
        }
      if (g.has_stats) {
        s = row4_sum(s);
        q = row4_sum(q);
        if (lane < 16 && col < N) {
          red[wm * LDC + col - cbase] += s;
          red[(2 + wm) * LDC + col - cbase] += q;
        }
      }
    }
    if (bpipe && ch + 1 < ch_end) {  // the other buffer was last read by chunk ch-1
      commit_b(Bs + ((ch + 1 - ch_begin) & 1) * RNB * LDA);
      if (ch + 2 < ch_end) fetch_b(ch + 2);
    }
    __syncthreads();
  }
// ---- write the staged tile: one linear stream when the rows are contiguous
  T* C = (T*)g.c;
  const int rows = min(BM, g.M - row0);
  if (ncols == N && g.ldc == N && (N & 7) == 0 && LDC == N) {
    const int nvec = rows * N / 8;
    T* dst = C + (size_t)row0 * N;
    for (int v = tid; v < nvec; v += 256) {
      float vals[8];
      const T* src = Cs + v * 8;
      if constexpr (sizeof(T) == 2) {
        uint4 raw = *reinterpret_cast<const uint4*>(src);
        if (!g.accumulate) { *reinterpret_cast<uint4*>(dst + v * 8) = raw; continue; }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = to_f<T>(src[j]);
      acc8m(dst + v * 8, 8, vals, g.accumulate);
    }
  } else {
    const int cv8 = cdiv(ncols, 8);
    const bool vec_ok = (g.ldc % 8) == 0;
    for (int v = tid; v < rows * cv8; v += 256) {
      const int r = v / cv8, cv = (v - r * cv8) * 8;
      const int nn = ncols - cv;
      float vals[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = to_f<T>(Cs[r * LDC + cv + j]);
      T* dst = C + (size_t)(row0 + r) * g.ldc + cbase + cv;
      if (vec_ok) {
        acc8m(dst, nn, vals, g.accumulate);
      } else {
        for (int j = 0; j < 8 && j < nn; ++j) dst[j] = from_f<T>(g.accumulate ? to_f<T>(dst[j]) + vals[j] : vals[j]);
      }
    }
  }
  }  // row tiles
  __syncthreads();
  if (cur_seg >= 0 && g.has_stats)
    for (int c = tid; c < ncols; c += 256) {
      stat_put(g.stats.sum[cur_seg], cbase + c, (double)(red[c] + red[LDC + c]));
      stat_put(g.stats.sq[cur_seg], cbase + c, (double)(red[2 * LDC + c] + red[3 * LDC + c]));
    }
}

// ------------------------------------------------------------------ weight gradient
struct WgradArgs {
  const void* a;
  const void* dy;
  float* dw;
  float* db;
  float* part;  // non-null: per-split partials [split][N][K] then [split][N] (no atomics)
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

// bf16 weight gradient with natural-layout LDS images and gfx950 transposed LDS reads.
// dW[n][k] = sum_m dY[m][n] * v(A)[m][k]: both operands are m-major in HBM, and the MFMA
// wants 8 consecutive m per lane, so the [m][n] / [m][k] tiles are written to LDS exactly as
// they arrive (16-byte stores) and read with ds_read_b64_tr_b16, which hands lane i of each
// 16-lane group column i of 4 rows.  64-row stages, double-buffered in LDS with the next
// stage prefetched into registers: one barrier per stage.
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef short v8s_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s_t lds_v4s;

__device__ __forceinline__ bf16x8_t tr_frag(const uint16_t* img, int ldm, int r0, int c0) {
  const int lane = threadIdx.x & 63, q = (lane & 15) >> 2, p = lane & 3;
  const uint16_t* a = img + (r0 + 8 * (lane >> 4) + q) * ldm + c0 + 4 * p;
  const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)a);
  const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a + 4 * ldm));
  const v8s_t c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8_t, c);
}

constexpr int WT_BM = 64, WT_LDM = 64 + 8;  // WT_BM: the unit the row splits are sized in

// BM rows per stage (one barrier each), PF stages in flight in registers ahead of the one being
// committed.  A block's stage chain is latency-bound on the mid-M shapes (~1.2 us per 64-row
// stage at 2 in flight, whatever the tile count: profiles/r03ab_wgrad_plan_sweep.txt), so more
// bytes in flight per block shorten it without adding splits (= fp32 atomic bytes).
// ACT (LAZY): the activation as a compile-time case (0 none, 1 swish), as k_gemm_s
template <bool LAZY, int BM = 64, int PF = 2, int ACT = 0>
__global__ __launch_bounds__(256) void k_wgrad_tr(WgradArgs g) {
  static_assert(BM % 64 == 0 && PF >= 1, "stage rows: multiple of 64");
  constexpr int HR = BM / 32;  // rows per thread per stage (32 rows per pass of the 256 threads)
  __shared__ __attribute__((aligned(16))) uint16_t Ds[2][BM * WT_LDM];
  __shared__ __attribute__((aligned(16))) uint16_t Xs[2][BM * WT_LDM];
  __shared__ float2 xf[EDET_MAX_SEG][64];
  __shared__ float dbred[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int ntiles = g.ntn * g.ntk;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lid / ntiles, tile = lid - split * ntiles;
  const int tn = tile / g.ntk, tk = tile - tn * g.ntk;
  const int n0 = tn * 64, kk0 = tk * 64;
  const int m_begin = split * g.rows_per;
  const int m_end = min(g.M, m_begin + g.rows_per);
  const bool do_db = (g.db != nullptr) && tk == 0;
  const uint16_t* DY = (const uint16_t*)g.dy;
  const uint16_t* A = (const uint16_t*)g.a;
  if constexpr (LAZY) {
    for (int e = tid; e < g.pyr.nseg * 64; e += 256) {
      const int sg = e >> 6, k = kk0 + (e & 63);
      xf[sg][e & 63] = (k < g.K) ? bn_affine(g.lz.bn, sg, k, 1.f / (float)seg_rows(g.pyr, sg)) : make_float2(1.f, 0.f);
    }
  }
  // each thread moves rows (tid>>3) + 32h, 8-column vector (tid&7)*8 of both tiles
  const int lr = tid >> 3, lc = (tid & 7) * 8;
  struct Stage {
    uint4 rd[HR], rx[HR];
    int rseg[HR];
    uint4 rg[LAZY ? HR : 1][2];  // LAZY: the SE gate of the row's image, this thread's 8 columns
  };
  // Branch-free fetches: a dead row (past the range or in a segment's padding) loads a live row
  // of the block and a column vector past the row loads the row's last vector, and commit zeroes
  // both.  A vector straddling N (or K) is loaded whole: lda / lddy % 8 == 0 keeps it inside the
  // row, and its columns >= N (>= K) only reach dW rows (columns) that are never stored.  With
  // every load unconditional the compiler's wait before a commit counts only that stage's loads
  // (loads under branches made it wait for every stage in flight: s_waitcnt vmcnt(0)).
  const bool dcol = n0 + lc < g.N, xcol = kk0 + lc < g.K;
  const int dc = min(n0 + lc, g.lddy - 8), xc = min(kk0 + lc, g.lda - 8);
  // LAZY with an SE gate (one segment, the host requires it): the gate vector of each row's
  // image is fetched with the row, by a range-checked buffer load (no gate: an empty range, the
  // load reads zeros and is not used).  A gate load in the commit, under the per-image branch,
  // made every commit wait for all the stages in flight (s_waitcnt vmcnt(0), scripts/wait_scan.py).
  const bool has_gate = LAZY && g.lz.gate != nullptr;
  const auto rs_gate = buf_rsrc(LAZY ? g.lz.gate : nullptr, has_gate ? (long)g.pyr.batch * g.K * 4 : 0);
  const int hw0 = g.pyr.H[0] * g.pyr.W[0], off0 = g.pyr.row_off[0];
  auto fetch = [&](Stage& S, int m0) {
#pragma unroll
    for (int h = 0; h < HR; ++h) {
      const int row = m0 + lr + 32 * h;
      int send;
      const int sg = seg_of_row_end(g.pyr, row, send);
      const bool live = row < m_end && row < send;
      S.rseg[h] = live ? sg : -1;
      const size_t r = live ? row : m_begin;
      S.rd[h] = *reinterpret_cast<const uint4*>(DY + r * g.lddy + dc);
      S.rx[h] = *reinterpret_cast<const uint4*>(A + r * g.lda + xc);
      if constexpr (LAZY) {
        const int img = ((int)r - off0) / hw0;
        const uint32_t go = buf_off(has_gate && xcol, (uint32_t)((img * g.K + kk0 + lc) * 4));
        S.rg[h][0] = buf_ld16(rs_gate, go);
        S.rg[h][1] = buf_ld16(rs_gate, go + 16);
      }
    }
  };
  auto zsel = [](bool keep, uint4 v) {
    return make_uint4(keep ? v.x : 0u, keep ? v.y : 0u, keep ? v.z : 0u, keep ? v.w : 0u);
  };
  // (branch-free: dead rows and columns past K are transformed like live ones and selected out)
  auto commit = [&](const Stage& S, int buf, int m0) {
#pragma unroll
    for (int h = 0; h < HR; ++h) {
      const int r = lr + 32 * h;
      *reinterpret_cast<uint4*>(&Ds[buf][r * WT_LDM + lc]) = zsel(S.rseg[h] >= 0 && dcol, S.rd[h]);
      uint4 x;
      if constexpr (LAZY) {
        const int sg = max(S.rseg[h], 0);
        const bool keep = S.rseg[h] >= 0 && xcol;
        const uint16_t* t = reinterpret_cast<const uint16_t*>(&S.rx[h]);
        const float4 g0 = __builtin_bit_cast(float4, S.rg[h][0]), g1 = __builtin_bit_cast(float4, S.rg[h][1]);
        const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        uint16_t o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float2 a = xf[sg][lc + j];
          float u = to_f<uint16_t>(t[j]) * a.x + a.y;
          if constexpr (ACT == 1) u = swishf_(u);
          if (has_gate) u *= gv[j];
          o[j] = from_f<uint16_t>(keep && kk0 + lc + j < g.K ? u : 0.f);
        }
        x = *reinterpret_cast<uint4*>(o);
      } else {
        x = zsel(S.rseg[h] >= 0 && xcol, S.rx[h]);
      }
      *reinterpret_cast<uint4*>(&Xs[buf][r * WT_LDM + lc]) = x;
    }
  };

  floatx4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  if constexpr (LAZY) __syncthreads();  // xf tables
  // stage t sits in LDS buffer t & 1; stage t + 1 is in register slot t % PF when stage t is
  // multiplied, and its slot is refilled with stage t + 1 + PF right after its commit
  // Every fetch / commit / stage runs unconditionally (stages past the block's rows are all
  // dead rows: zeros in LDS, nothing added): a fetch under a branch leaves the compiler's
  // wait-count merge pessimistic, and each commit then waited for the stages behind it too.
  Stage S[PF];
  fetch(S[0], m_begin);
  commit(S[0], 0, m_begin);
#pragma unroll
  for (int p = 0; p < PF; ++p) fetch(S[p], m_begin + (p + 1) * BM);
  __syncthreads();
  int t = 0;
  auto iter = [&](Stage& R, int m0, int buf) {
#pragma unroll
    for (int ks = 0; ks < BM; ks += 32) {
      bf16x8_t af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tr_frag(Ds[buf], WT_LDM, ks, wn * 32 + i * 16);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tr_frag(Xs[buf], WT_LDM, ks, wk * 32 + j * 16);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (do_db) {
      const uint16_t* col = &Ds[buf][(wave * (BM / 4)) * WT_LDM + lane];
#pragma unroll
      for (int m = 0; m < BM / 4; ++m) dbacc += to_f<uint16_t>(col[m * WT_LDM]);
    }
    commit(R, buf ^ 1, m0 + BM);
    fetch(R, m0 + (PF + 1) * BM);
    __syncthreads();
    ++t;
  };
  for (int m0 = m_begin; m0 < m_end; m0 += PF * BM) {
#pragma unroll
    for (int p = 0; p < PF; ++p)  // (an even PF keeps the LDS buffer a compile-time constant)
      iter(S[p], m0 + p * BM, PF % 2 == 0 ? (p & 1) : (t & 1));
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int k = kk0 + wk * 32 + j * 16 + (lane & 15);
        if (n < g.N && k < g.K) {
          if (g.part) g.part[((size_t)split * g.N + n) * g.K + k] = acc[i][j][r];
          else atomicAdd(g.dw + (size_t)n * g.K + k, acc[i][j][r]);
        }
      }
  if (do_db) {
    dbred[wave][lane] = dbacc;
    __syncthreads();
    if (tid < 64 && n0 + tid < g.N) {
      const float v = dbred[0][tid] + dbred[1][tid] + dbred[2][tid] + dbred[3][tid];
      if (g.part) g.part[(size_t)gridDim.x / (g.ntn * g.ntk) * g.N * g.K + (size_t)split * g.N + n0 + tid] = v;
      else atomicAdd(g.db + n0 + tid, v);
    }
  }
}

// ------------------------------------------------------------------ wave-streaming weight gradient
// dW[n][k] = sum_m dY[m][n] * A[m][k] (+ db[n] = sum_m dY[m][n]) for a plain bf16 A.
//
// The product is a reduction over the very long m axis of two m-major operands.  Each wave
// owns the whole 16FN x 16FK output tile of its block and streams its own 32-row groups: the
// group's dY and A rows arrive as 16-byte vectors (one row of the tile = 2(FN+FK) vectors, the
// wave's 64 lanes cover 32 rows x that), are written to the wave's private LDS image as they
// are, and read back m-contiguous with gfx950's transposing ds_read_b64_tr_b16 as MFMA
// fragments: FN x FK v_mfma_f32_16x16x32_bf16 per group, plus FN against an all-ones fragment
// for the bias gradient.  No block barrier in the row loop; the next WS_PF groups' vectors are
// in flight while a group is multiplied.  Each element of dY and A is read once per tile
// (once overall when the tile covers N x K), the 4 waves' partial tiles are folded in LDS in a
// fixed order and leave the block once, as plain stores into the caller's split-partials
// workspace (one fixed-order sum pass after) or as fp32 atomics without a workspace.
struct WgsArgs {
  const uint16_t* a;
  const uint16_t* dy;
  float* dw;
  float* db;
  float* part;  // [split][N][K] then [split][N], or null: atomics into dw / db
  edet_pyramid pyr;
  int lda, lddy, M, K, N;
  int ntk, splits, gpb, ngrp;
};

constexpr int WS_PF = 2;  // groups in flight ahead of the one being multiplied

template <int FN, int FK>
__global__ __launch_bounds__(256) void k_wgs(WgsArgs g) {
  constexpr int CW = 2 * (FN + FK);        // 16-byte vectors per tile row
  constexpr int VPL = FN + FK;             // vectors per lane per 32-row group (32 * CW / 64)
  constexpr int LDM = 16 * (FN + FK) + 8;  // LDS image row (bf16), padded
  extern __shared__ __attribute__((aligned(16))) uint16_t wsm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = lid / g.splits, split = lid - tile * g.splits;
  const int tn = tile / g.ntk, tk = tile - tn * g.ntk;
  const int n0 = tn * 16 * FN, k0 = tk * 16 * FK;
  const bool do_db = g.db != nullptr && tk == 0;
  uint16_t* img = wsm + wave * 32 * LDM;
  const int gbeg = split * g.gpb, gend = min(g.ngrp, gbeg + g.gpb);

  // this lane's vectors of a group: (row, vector-in-row) pairs are compile-time per slot
  auto fetch = [&](int grp, uint4* v) {
    int seg = 0;
    for (int s = 1; s < g.pyr.nseg; ++s)
      if (grp * 32 >= g.pyr.row_off[s]) seg = s;
    const int rend = g.pyr.row_off[seg] + seg_rows(g.pyr, seg);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int e = lane + 64 * i, r = e / CW, c = e - r * CW;
      const int row = grp * 32 + r;
      const bool live = grp < gend && row < rend;
      const uint16_t* p;
      bool ok;
      if (c < 2 * FN) {
        const int col = n0 + 8 * c;
        ok = live && col < g.lddy;
        p = g.dy + (size_t)row * g.lddy + col;
      } else {
        const int col = k0 + 8 * (c - 2 * FN);
        ok = live && col < g.K;
        p = g.a + (size_t)row * g.lda + col;
      }
      // select-predicated address: the load is issued unconditionally (a load inside a
      // divergent branch is waited on inside it)
      const uint4 t = *reinterpret_cast<const uint4*>(ok ? p : g.dy);
      v[i] = ok ? t : make_uint4(0, 0, 0, 0);
    }
  };

  floatx4 acc[FN][FK], accb[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    accb[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < FK; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u));

  uint4 pre[WS_PF][VPL];
#pragma unroll
  for (int u = 0; u < WS_PF; ++u) fetch(gbeg + wave + 4 * u, pre[u]);
  for (int grp = gbeg + wave; grp < gend; grp += 4) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int e = lane + 64 * i, r = e / CW, c = e - r * CW;
      *reinterpret_cast<uint4*>(img + r * LDM + 8 * c) = pre[0][i];
    }
#pragma unroll
    for (int u = 0; u + 1 < WS_PF; ++u)
#pragma unroll
      for (int i = 0; i < VPL; ++i) pre[u][i] = pre[u + 1][i];
    fetch(grp + 4 * WS_PF, pre[WS_PF - 1]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bf16x8_t fa[FN], fb[FK];
#pragma unroll
    for (int i = 0; i < FN; ++i) fa[i] = tr_frag(img, LDM, 0, 16 * i);
#pragma unroll
    for (int j = 0; j < FK; ++j) fb[j] = tr_frag(img, LDM, 0, 16 * (FN + j));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < FN; ++i) {
#pragma unroll
      for (int j = 0; j < FK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (do_db) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accb[i], 0, 0, 0);
    }
  }

  // fold the 4 waves' tiles in LDS (fixed order: ((w0 + w1) + (w2 + w3))), lane-major slots
  __syncthreads();
  float* red = reinterpret_cast<float*>(wsm);  // [2][FN*FK+FN][4][64]
  constexpr int NV = FN * FK + FN;
  auto put = [&](int slot) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
#pragma unroll
      for (int j = 0; j < FK; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[((slot * NV + i * FK + j) * 4 + r) * 64 + lane] = acc[i][j][r];
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((slot * NV + FN * FK + i) * 4 + r) * 64 + lane] = accb[i][r];
    }
  };
  auto add = [&](int slot) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
#pragma unroll
      for (int j = 0; j < FK; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += red[((slot * NV + i * FK + j) * 4 + r) * 64 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) accb[i][r] += red[((slot * NV + FN * FK + i) * 4 + r) * 64 + lane];
    }
  };
  if (wave >= 2) put(wave - 2);
  __syncthreads();
  if (wave < 2) add(wave);
  __syncthreads();
  if (wave == 1) put(0);
  __syncthreads();
  if (wave != 0) return;
  add(0);
#pragma unroll
  for (int i = 0; i < FN; ++i) {
#pragma unroll
    for (int j = 0; j < FK; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 16 * i + 4 * (lane >> 4) + r, k = k0 + 16 * j + (lane & 15);
        if (n < g.N && k < g.K) {
          if (g.part) g.part[((size_t)split * g.N + n) * g.K + k] = acc[i][j][r];
          else atomicAdd(g.dw + (size_t)n * g.K + k, acc[i][j][r]);
        }
      }
    if (do_db && (lane & 15) == 0)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 16 * i + 4 * (lane >> 4) + r;
        if (n < g.N) {
          if (g.part) g.part[(size_t)g.splits * g.N * g.K + (size_t)split * g.N + n] = accb[i][r];
          else atomicAdd(g.db + n, accb[i][r]);
        }
      }
  }
}

struct WgsShape {
  int fn, fk;
};
// instantiated tiles (16FN x 16FK outputs per block)
constexpr WgsShape WGS_SHAPES[] = {{1, 2}, {2, 2}, {2, 3}, {3, 2}, {6, 1}, {4, 4}, {2, 4}, {4, 2}, {3, 3}};
constexpr int WGS_NARROW = 5;  // the first five: the narrow tiles of the production plan

template <int FN, int FK>
static int launch_wgs(WgsArgs g, int grid, hipStream_t s) {
  constexpr int LDM = 16 * (FN + FK) + 8;
  const size_t stage = 4 * 32 * LDM * sizeof(uint16_t);
  const size_t red = 2 * (FN * FK + FN) * 4 * 64 * sizeof(float);
  const size_t lds = stage > red ? stage : red;
  EDET_LAUNCH((k_wgs<FN, FK>), dim3(grid), dim3(256), lds, s, g);
  return check_launch("edet wgrad");
}

static int dispatch_wgs(WgsArgs g, int fn, int fk, int grid, hipStream_t s) {
#define EDET_WGS_CASE(A, B) \
  if (fn == A && fk == B) return launch_wgs<A, B>(g, grid, s);
  EDET_WGS_CASE(1, 2) EDET_WGS_CASE(2, 2) EDET_WGS_CASE(2, 3) EDET_WGS_CASE(3, 2) EDET_WGS_CASE(6, 1)
  EDET_WGS_CASE(4, 4) EDET_WGS_CASE(2, 4) EDET_WGS_CASE(4, 2) EDET_WGS_CASE(3, 3)
#undef EDET_WGS_CASE
  set_error("wgrad: no tile %dx%d", fn, fk);
  return EDET_EUNSUPPORTED;
}

// the tile that moves the fewest bytes: each tile re-reads dY for every K tile and A for every
// N tile (N rounded to the tile's 16-column fragments), plus a small charge per fragment for
// the MFMA and LDS work of zero-padded columns
static WgsShape pick_wgs(int N, int K, bool wide) {
  const int FNt = cdiv(N, 16), FKt = cdiv(K, 16);
  WgsShape best{0, 0};
  double bc = 1e300;
  const int nshapes = wide ? (int)(sizeof(WGS_SHAPES) / sizeof(WGS_SHAPES[0])) : WGS_NARROW;
  for (int si = 0; si < nshapes; ++si) {
    const WgsShape& t = WGS_SHAPES[si];
    const int ntn = cdiv(FNt, t.fn), ntk = cdiv(FKt, t.fk);
    const double bytes = (double)ntk * 16 * t.fn * ntn + (double)ntn * 16 * t.fk * ntk;
    const double frags = (double)ntn * ntk * t.fn * t.fk;
    const double cost = bytes + 6.0 * frags;
    if (cost < bc) { bc = cost; best = t; }
  }
  return best;
}

// ------------------------------------------------------------------ B-resident GEMM
// Persistent kernel for the memory-bound 1x1 convs.  Each block loads its column group of the
// weight B [NG][KP] into LDS ONCE, then streams A through the chip in chunks of R rows x KC
// columns (~16 KB): chunk q+1 is fetched global -> registers (raw values, plus the SE gate
// values it will need) while chunk q is multiplied, then transformed (lazy BN / swish / gate)
// into the other LDS buffer; one barrier per chunk.  Without B traffic the per-CU request
// stream is only A (the previous kernels re-read B from L2 for every 32-128 row tile, and the
// counters showed them parked on memory for ~65 % of the wave cycles).
//   case S (!KSTREAM): the chunk holds whole rows (KC = KP <= 256), R = 64..256 rows; every
//     64-row tile is multiplied against the group's columns in 64-column sub-chunks.
//   case L (KSTREAM): R = 64, K walked in KC = 128 slices with the accumulators kept; NG =
//     32 * FN columns per group (B [NG][KP] still resident).
// Output: each wave stages its 32 x 16*FN accumulator tile in a private LDS patch and writes
// it back as 16-byte row vectors (no block barrier).  BN statistics: per-block fp32 partials
// in LDS with one owner lane each, flushed as fp64 atomics once per segment.
struct PwPlan {
  int R, KC, KP, nkc, NG, ngroups, nrg, LDA, LDB, nsub, NGtot;
};

constexpr int PW_NV = 8;  // max 16-byte A vectors per thread per chunk

template <typename T, int FN, bool KSTREAM, bool LAZY, bool GATE = false>
__global__ __launch_bounds__(256) void k_pwb(GemmArgs g, PwPlan p) {
  static_assert(!GATE || LAZY, "gate: lazy A only");
  using V = typename std::conditional<sizeof(T) == 2, uint4, float4>::type;
  constexpr int VW = sizeof(T) == 2 ? 1 : 2;
  constexpr int CWLD = 16 * FN + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* Bs = reinterpret_cast<T*>(smem);                  // [NG][LDB]
  T* As = Bs + (size_t)p.NG * p.LDB;                    // [2][R][LDA]
  T* Cw = As + 2 * (size_t)p.R * p.LDA;                 // [4 waves][32][CWLD]
  float* red = reinterpret_cast<float*>(Cw + 4 * 32 * CWLD);  // [sum|sq][wm][NGtot]
  float* bias_s = red + 4 * p.NGtot;                          // [NGtot] (a bias load in the
  // epilogue would be waited for behind the next chunk's prefetch)
  float2* xf = reinterpret_cast<float2*>(bias_s + p.NGtot);   // [nseg][KP] (LAZY)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = w % p.ngroups, G = gridDim.x / p.ngroups;
  const int rg0 = w / p.ngroups;
  if (rg0 >= p.nrg) return;
  const int col_base = grp * p.NG;
  const int K = g.K, N = g.N, M = g.M;

  // ---- resident B (this group's columns, zero past N and K), stats partials, BN affine
  {
    const T* B = (const T*)g.b;
    const int kvb = p.KP / 8;
    for (int v = tid; v < p.NG * kvb; v += 256) {
      const int n = v / kvb, kv = (v - n * kvb) * 8, gn = col_base + n;
      T* dst = Bs + (size_t)n * p.LDB + kv;
      if (gn < N && kv < K) cp8(dst, B + (size_t)gn * g.ldb + kv, K - kv);
      else zero8(dst);
    }
    for (int c = tid; c < 4 * p.NGtot; c += 256) red[c] = 0.f;
    for (int c = tid; c < p.NGtot; c += 256) bias_s[c] = (g.bias && col_base + c < N) ? g.bias[col_base + c] : 0.f;
    if constexpr (LAZY) {
      for (int s = 0; s < g.pyr.nseg; ++s) {
        const float inv = 1.f / (float)seg_rows(g.pyr, s);
        for (int k = tid; k < p.KP; k += 256) xf[s * p.KP + k] = k < K ? bn_affine(g.lz.bn, s, k, inv) : make_float2(0.f, 0.f);
      }
    }
  }

  const int KV = p.KC / 8;
  const int nvec = p.R * KV;
  const int nq = ((p.nrg - 1 - rg0) / G + 1) * p.nkc;
  const T* A = (const T*)g.a;
  constexpr bool has_gate = GATE;  // (the gate vectors cost 64 registers: their own instance)
  V ra[PW_NV][VW];
  float4 gr[GATE ? PW_NV : 1][2];

  // Branch-free fetch: range-checked loads (rows past M, columns past K and the gate of a dead
  // element read zeros; a launch without a gate reads through an empty range).  Loads under
  // branches merged into registers that live across the chunk loop: the compiler waited for
  // each one where it was issued.
  const auto rs_gate = buf_rsrc(GATE ? g.lz.gate : nullptr, GATE ? (long)g.pyr.batch * K * 4 : 0);
  auto fetch = [&](int q) {
    const int rg = rg0 + (q / p.nkc) * G, kc = q % p.nkc;
    const int rbase = rg * p.R;
    int seg = 0, seg_off = 0, hw = 1;
    if (has_gate) { seg = seg_of_row(g.pyr, rbase); seg_off = g.pyr.row_off[seg]; hw = g.pyr.H[seg] * g.pyr.W[seg]; }
    const auto rs_a = buf_rsrc(A + (size_t)rbase * g.lda, (long)min(p.R, M - rbase) * g.lda * (long)sizeof(T));
#pragma unroll
    for (int u = 0; u < PW_NV; ++u) {
      const int v = tid + u * 256;
      const int r = v / KV, kv = (v - r * KV) * 8;
      const int grow = rbase + r, gk = kc * p.KC + kv;
      const bool ok = v < nvec && gk < K;
      const uint32_t off = buf_off(ok, (uint32_t)((r * g.lda + gk) * (int)sizeof(T)));
#pragma unroll
      for (int ww = 0; ww < VW; ++ww) ra[u][ww] = __builtin_bit_cast(V, buf_ld16(rs_a, off + 16 * ww));
      if constexpr (GATE) {
        const uint32_t goff = buf_off(ok && grow < M, (uint32_t)((((grow - seg_off) / hw) * K + gk) * 4));
        gr[u][0] = __builtin_bit_cast(float4, buf_ld16(rs_gate, goff));
        gr[u][1] = __builtin_bit_cast(float4, buf_ld16(rs_gate, goff + 16));
      }
    }
  };
  auto commit = [&](int q, int buf) {
    const int rg = rg0 + (q / p.nkc) * G, kc = q % p.nkc;
    const int rbase = rg * p.R;
    const int seg = LAZY ? seg_of_row(g.pyr, rbase) : 0;
    T* Ab = As + (size_t)buf * p.R * p.LDA;
#pragma unroll
    for (int u = 0; u < PW_NV; ++u) {
      const int v = tid + u * 256;
      if (v >= nvec) break;
      const int r = v / KV, kv = (v - r * KV) * 8;
      T* dst = Ab + (size_t)r * p.LDA + kv;
      if constexpr (LAZY) {
        const int grow = rbase + r, gk = kc * p.KC + kv;
        const bool live = grow < M && gk < K;
        const T* e = reinterpret_cast<const T*>(&ra[u][0]);
        const float4 g0 = GATE ? gr[u][0] : make_float4(1.f, 1.f, 1.f, 1.f);
        const float4 g1 = GATE ? gr[u][1] : make_float4(1.f, 1.f, 1.f, 1.f);
        const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        const float2* af = xf + seg * p.KP + (live ? gk : 0);
        float vals[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = lazy_apply(to_f<T>(e[j]), af[j], g.lz.act);
          if (has_gate) x *= gv[j];
          vals[j] = live ? x : 0.f;
        }
        st8(dst, vals);
      } else {
#pragma unroll
        for (int ww = 0; ww < VW; ++ww) reinterpret_cast<V*>(dst)[ww] = ra[u][ww];
      }
    }
  };

  // ---- MFMA over k in [0, kn) of A rows (a_row0 ..) x B rows (b_row0 ..) at B column kb0
  auto mma = [&](floatx4 (&acc)[2][FN], const T* Ab, int a_row0, int b_row0, int kb0, int kn) {
    const T* ap = Ab + (size_t)(a_row0 + wm * 32 + (lane & 15)) * p.LDA;
    const T* bp = Bs + (size_t)(b_row0 + wn * 16 * FN + (lane & 15)) * p.LDB + kb0;
    for (int ks = 0; ks < kn; ks += 32) {
      if constexpr (sizeof(T) == 2) {
        bf16x8_t af[2], bfr[FN];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = lds_frag_bf16(ap + (size_t)i * 16 * p.LDA + ks + 8 * (lane >> 4));
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = lds_frag_bf16(bp + (size_t)j * 16 * p.LDB + ks + 8 * (lane >> 4));
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      } else {
#pragma unroll
        for (int s4 = 0; s4 < 8; ++s4) {
          float af[2], bfr[FN];
#pragma unroll
          for (int i = 0; i < 2; ++i) af[i] = ap[(size_t)i * 16 * p.LDA + ks + 4 * s4 + (lane >> 4)];
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[j] = bp[(size_t)j * 16 * p.LDB + ks + 4 * s4 + (lane >> 4)];
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
  };

  // ---- epilogue of one wave tile: rows row0 + wm*32 .., group-local columns cl0 + wn*16*FN ..
  T* cw = Cw + (size_t)wave * 32 * CWLD;
  T* C = (T*)g.c;
  auto epilogue = [&](floatx4 (&acc)[2][FN], int row0, int cl0, int seg_end) {
    const int wrow0 = row0 + wm * 32;
    const int wcl0 = cl0 + wn * 16 * FN;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cl = wcl0 + j * 16 + (lane & 15);
      const float bv = bias_s[cl];
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = i * 16 + (lane >> 4) * 4 + r;
          const float v = acc[i][j][r] + bv;
          cw[rl * CWLD + j * 16 + (lane & 15)] = from_f<T>(v);
          if (wrow0 + rl < seg_end) { s += v; q += v * v; }
        }
      if (g.has_stats) {
        s = row4_sum(s);
        q = row4_sum(q);
        if (lane < 16) {  // sole owner of (wm, cl)
          red[(0 * 2 + wm) * p.NGtot + cl] += s;
          red[(1 * 2 + wm) * p.NGtot + cl] += q;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int VPR = 2 * FN;  // 8-element vectors per tile row
#pragma unroll
    for (int e = lane; e < 32 * VPR; e += 64) {
      const int rr = e / VPR, cv = (e - rr * VPR) * 8;
      const int grow = wrow0 + rr, gcol = col_base + wcl0 + cv;
      if (grow < M && gcol < N) {
        float vals[8];
        const T* src = cw + rr * CWLD + cv;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) vals[jj] = to_f<T>(src[jj]);
        acc8m(C + (size_t)grow * g.ldc + gcol, N - gcol, vals, g.accumulate);
      }
    }
  };
  auto flush = [&](int seg) {
    if (!g.has_stats || seg < 0 || lane >= 16) return;
    for (int sub = 0; sub < p.nsub; ++sub)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int cl = sub * 64 + wn * 16 * FN + j * 16 + lane;
        const int col = col_base + cl;
        if (col < N && cl < p.NGtot) {
          float& rs = red[(0 * 2 + wm) * p.NGtot + cl];
          float& rq = red[(1 * 2 + wm) * p.NGtot + cl];
          stat_put(g.stats.sum[seg], col, (double)rs);
          stat_put(g.stats.sq[seg], col, (double)rq);
          rs = 0.f;
          rq = 0.f;
        }
      }
  };

  floatx4 acc[2][FN];
  int cur_seg = -1;
  fetch(0);
  __syncthreads();  // B, affine tables and partials are in place
  commit(0, 0);
  __syncthreads();
  for (int q = 0; q < nq; ++q) {
    const int buf = q & 1;
    const bool more = q + 1 < nq;
    if (more) fetch(q + 1);
    const int rg = rg0 + (q / p.nkc) * G, kc = q % p.nkc;
    const int rbase = rg * p.R;
    const int seg = seg_of_row(g.pyr, rbase);
    const int seg_end = g.pyr.row_off[seg] + seg_rows(g.pyr, seg);
    if (seg != cur_seg) {
      flush(cur_seg);
      cur_seg = seg;
    }
    const T* Ab = As + (size_t)buf * p.R * p.LDA;
    if constexpr (!KSTREAM) {
      for (int t = 0; t < p.R / 64; ++t) {
        const int row0 = rbase + t * 64;
        if (row0 >= M) break;
        for (int sub = 0; sub < p.nsub; ++sub) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
          mma(acc, Ab, t * 64, sub * 64, 0, p.KP);
          epilogue(acc, row0, sub * 64, seg_end);
        }
      }
    } else {
      if (kc == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
      mma(acc, Ab, 0, 0, kc * p.KC, p.KC);
      if (kc == p.nkc - 1) epilogue(acc, rbase, 0, seg_end);
    }
    if (more) commit(q + 1, buf ^ 1);
    __syncthreads();
  }
  flush(cur_seg);
}

static size_t pw_lds(const PwPlan& p, int FN, int nseg, bool lazy, int es) {
  return (size_t)p.NG * p.LDB * es + 2 * (size_t)p.R * p.LDA * es + 4 * 32 * (16 * FN + 8) * (size_t)es +
         5 * (size_t)p.NGtot * 4 + (lazy ? (size_t)nseg * p.KP * 8 : 0);
}

// Plan the B-resident launch; false when the shape does not fit (caller falls back).
static bool pw_plan(const GemmArgs& g, bool lazy, int es, PwPlan& p, int& FN, bool& kstream) {
  const bool gate = lazy && g.lz.gate != nullptr;
  const int nseg = g.pyr.nseg;
  p.KP = cdiv(g.K, 32) * 32;
  kstream = p.KP > (gate ? 128 : 256);
  constexpr size_t CAP = 150 * 1024, PAIR = 78 * 1024;  // one / two blocks per CU
  if (!kstream) {
    p.KC = p.KP;
    p.nkc = 1;
    int R = 64;
    while (R < 256 && 2 * R * p.KP <= 8192) R *= 2;
    if (nseg > 1 && R > 128) R = 128;  // chunks never straddle a (128-aligned) segment start
    p.R = R;
    p.LDA = p.LDB = p.KP + 8;
    FN = 2;
    const int nch = cdiv(g.N, 64);
    // fewest column groups whose LDS image fits; two blocks per CU preferred up to 4 groups
    int best = -1;
    for (int ng = 1; ng <= nch; ++ng) {
      const int cps = cdiv(nch, ng);
      PwPlan t = p;
      t.NG = t.NGtot = cps * 64;
      t.nsub = cps;
      const size_t l = pw_lds(t, FN, nseg, lazy, es);
      if (l <= PAIR && ng <= 4) { best = ng; break; }
      if (l <= CAP && best < 0) best = ng;
      if (l <= CAP && ng > 4) break;
    }
    if (best < 0) return false;
    const int cps = cdiv(nch, best);
    p.NG = p.NGtot = cps * 64;
    p.nsub = cps;
    p.ngroups = cdiv(nch, cps);
  } else {
    p.KC = 128;
    p.KP = cdiv(g.K, p.KC) * p.KC;
    p.nkc = p.KP / p.KC;
    p.R = 64;
    p.LDA = p.KC + 8;
    p.LDB = p.KP + 8;
    p.nsub = 1;
    FN = 2;
    p.NG = p.NGtot = 64;
    if (pw_lds(p, FN, nseg, lazy, es) > CAP || g.N <= 32) {
      FN = 1;
      p.NG = p.NGtot = 32;
      if (pw_lds(p, FN, nseg, lazy, es) > CAP) return false;
    }
    p.ngroups = cdiv(g.N, p.NG);
  }
  p.nrg = cdiv(g.M, p.R);
  return true;
}

template <typename T, int FN, bool KS, bool LAZY>
static int launch_pwb(const GemmArgs& g, const PwPlan& p, hipStream_t s) {
  const size_t lds = pw_lds(p, FN, g.pyr.nseg, LAZY, sizeof(T));
  const int per_cu = lds <= 78 * 1024 ? 2 : 1;
  const long want = (long)256 * per_cu;
  long rows = std::min<long>(p.nrg, std::max<long>(1, want / p.ngroups));
  const int grid = (int)(rows * p.ngroups);
  if (LAZY && g.lz.gate) EDET_LAUNCH((k_pwb<T, FN, KS, LAZY, LAZY>), dim3(grid), dim3(256), lds, s, g, p);
  else EDET_LAUNCH((k_pwb<T, FN, KS, LAZY>), dim3(grid), dim3(256), lds, s, g, p);
  return check_launch("edet pwb");
}

template <typename T, bool LAZY>
static int dispatch_pwb(const GemmArgs& g, hipStream_t s, bool& done) {
  PwPlan p;
  int FN;
  bool ks;
  done = false;
  if (g.ldc % 8 != 0 || g.lda % 8 != 0 || g.K % 8 != 0) return EDET_OK;  // 16-byte row vectors
  if (g.M == 0 || !pw_plan(g, LAZY, sizeof(T), p, FN, ks)) return EDET_OK;
  // measured per shape against the A-resident / K-loop kernels (scripts/kbench.py): the
  // B-resident form wins for wide outputs over short rows, where those re-stage B per tile
  // (class predict 224 -> 104 us); the K-streamed variant re-reads and re-transforms A per
  // column group and loses
  const int KP = cdiv(g.K, 32) * 32;
  const bool lazy_in = LAZY;
  // D4+ (224-channel BiFPN and heads): K = 224 into N >= 192 also wins B-resident (the A-resident
  // form holds one block per CU there and re-stages B per row tile: D4 conv1x1 18.9 -> 17.7 ms per
  // step in kbench, r03t; wherever the plan fits, D0 lost 0.5 ms)
  const bool wide224 = g.N >= 192 && KP > 192 && KP <= 224;
  if (!wide224 && (ks || !(lazy_in ? (g.N >= 192 && KP <= 96) : (g.N >= 128 && KP <= 192)))) return EDET_OK;
  // except the stage-6 expand dgrad (8192 x 192 -> 1152): the A-resident form is faster there
  // (90 -> 63 us for its three calls, kbench round 2)
  if (g.M <= 8192 && g.N >= 1024) return EDET_OK;
  done = true;
  if (!ks) return launch_pwb<T, 2, false, LAZY>(g, p, s);
  if (FN == 2) return launch_pwb<T, 2, true, LAZY>(g, p, s);
  return launch_pwb<T, 1, true, LAZY>(g, p, s);
}

// the B-resident plan without the per-shape preference above (round-4 routing rules)
template <typename T, bool LAZY>
static int dispatch_pwb_forced(const GemmArgs& g, hipStream_t s, bool& done) {
  PwPlan p;
  int FN;
  bool ks;
  done = false;
  if (g.ldc % 8 != 0 || g.lda % 8 != 0 || g.K % 8 != 0) return EDET_OK;
  if (g.M == 0 || !pw_plan(g, LAZY, sizeof(T), p, FN, ks)) return EDET_OK;
  done = true;
  if (!ks) return launch_pwb<T, 2, false, LAZY>(g, p, s);
  if (FN == 2) return launch_pwb<T, 2, true, LAZY>(g, p, s);
  return launch_pwb<T, 1, true, LAZY>(g, p, s);
}

// ------------------------------------------------------------------ wave-streaming small-K GEMM
// For K <= 32 (the stage 0-1 convs: 2M x 16 -> 96, 524K x 24 -> 144, 2M x 32 -> 16) the
// GEMM is a pure stream: the outputs are 3-6x the inputs.  Every wave works alone, with no
// LDS and no barrier in the row loop: it keeps the weights as MFMA A-fragments in registers
// (W[n][k], 16 channels per fragment, K zero-padded to 32) and for each 16-row group loads its
// A rows straight into the B-fragment layout (lane = row, 8 consecutive k), applies the lazy
// BN/act/gate transform in registers, and issues one v_mfma_f32_16x16x32_bf16 per fragment.
// With A as the B operand each lane holds 4 consecutive output channels of one row: 8-byte
// stores, whole rows written by one wave back to back.  BN statistics stay in registers per
// lane until the end (one lane tree, one LDS pass and one fp64 atomic per channel per block).
constexpr int GS_PF = 2;  // row groups in flight ahead of the one being computed
// ACT (LAZY): the activation as a compile-time case (0 none, 1 swish).  The runtime test per
// element left the act = 0 instances slower than the swish ones (2M x 16 -> 96 with BN only:
// 152 -> 139 us, r05p)
template <typename T, int NF, int KS, bool LAZY, bool FOLD = false, int ACT = 0>
__global__ __launch_bounds__(256) void k_gemm_s(GemmArgs g) {
  // BN statistics: per wave and segment (a wave's groups ascend, so it meets each segment
  // once), summed over the block's waves in a fixed order at the end.  FOLD (one segment): the
  // same machinery carries the BN-backward sums (du, du * xhat) of the value y is the gradient of
  __shared__ float red[EDET_MAX_SEG][2][4][NF * 16];
  __shared__ float4 ftab[FOLD ? NF * 16 : 1];
  constexpr int LDW = NF * 16 + 8;  // wave-private output staging row (bf16), padded
  __shared__ __attribute__((aligned(16))) uint16_t stg[4][16 * LDW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint16_t* cw = stg[wave];
  const int kq = 8 * (lane >> 4);  // this lane's 8 k values
  // column slices (g.ncs > 1, the wide expand convs): block = (row range, slice of 16 NF
  // columns starting at nb0); every slice re-reads its rows' A (L2 hits: the slices of a row
  // range are neighbouring blocks)
  const int ncs = g.ncs > 1 ? g.ncs : 1;
  const int cs = blockIdx.x % ncs, rb = blockIdx.x / ncs, nrb = gridDim.x / ncs;
  const int nb0 = cs * NF * 16;
  const int K = g.K, N = min(g.N - nb0, NF * 16), M = g.M;
  const T* A = (const T*)g.a;
  const T* Wt = (const T*)g.b;
  T* Y = (T*)g.c;
  // weights: fragment (ks, f) holds W[16 f + (lane & 15)][32 ks + kq .. + 8]
  bf16x8_t wf[KS][NF];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int n = 16 * f + (lane & 15), k = 32 * ks + kq;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n < N && k < K) v = *reinterpret_cast<const uint4*>(Wt + (size_t)(nb0 + n) * g.ldb + k);
      wf[ks][f] = __builtin_bit_cast(bf16x8_t, v);
    }
  // bias in LDS (4 * NF registers per lane held it: at NF = 9 the difference between one and
  // two waves per SIMD)
  __shared__ __attribute__((aligned(16))) float bias_s[NF * 16];
  for (int n = threadIdx.x; n < NF * 16; n += 256) bias_s[n] = (g.bias && n < N) ? g.bias[nb0 + n] : 0.f;
  // the lazy BN affine of this lane's k values: registers for KS <= 2, LDS beyond (KS * 16
  // registers would cost the deep-K sliced forms their second wave per SIMD)
  constexpr bool AFR = KS <= 2;
  float2 af[AFR ? KS : 1][8];
  __shared__ float2 af_s[AFR ? 1 : KS * 32];
  if constexpr (LAZY) {
    const float inv = 1.f / (float)M;
    if constexpr (AFR) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          af[ks][j] = 32 * ks + kq + j < K ? bn_affine(g.lz.bn, 0, 32 * ks + kq + j, inv) : make_float2(1.f, 0.f);
    } else {
      for (int k = threadIdx.x; k < KS * 32; k += 256)
        af_s[k] = k < K ? bn_affine(g.lz.bn, 0, k, inv) : make_float2(1.f, 0.f);
    }
  }
  const int hw = g.pyr.H[0] * g.pyr.W[0];
  float ss[NF][4], sq[NF][4];
#pragma unroll
  for (int f = 0; f < NF; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) { ss[f][r] = 0.f; sq[f][r] = 0.f; }
  if (g.has_stats)
    for (int i = threadIdx.x; i < EDET_MAX_SEG * 2 * 4 * NF * 16; i += 256) (&red[0][0][0][0])[i] = 0.f;
  if constexpr (FOLD) {
    const float inv = 1.f / (float)seg_rows(g.pyr, 0);
    for (int c = threadIdx.x; c < NF * 16; c += 256)
      ftab[c] = c < N ? fold_table(g.fx.bn, 0, nb0 + c, inv) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  int cur_seg = -1, seg_end = g.has_stats ? 0 : M;
  // lanes sharing (lane >> 4) hold the same 4 channels of 16 different rows
  auto wflush = [&](int sg) {
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = ss[f][r], b = sq[f][r];
        a = row16_sum(a);
        b = row16_sum(b);
        if ((lane & 15) == 0) {
          red[sg][0][wave][16 * f + 4 * (lane >> 4) + r] = a;
          red[sg][1][wave][16 * f + 4 * (lane >> 4) + r] = b;
        }
        ss[f][r] = 0.f;
        sq[f][r] = 0.f;
      }
  };
  __syncthreads();  // red zeroed before any wave flushes; bias table in place
  // each block owns a contiguous range of 16-row groups (its waves interleave inside it), so
  // a block meets one pyramid level, rarely two: per-wave flushes and the block's fp64
  // atomics cover only the levels it touched (a grid-strided wave met a new level about once
  // per group and every block flushed all five)
  const int ngroups = (M + 15) / 16, gpb = (ngroups + nrb - 1) / nrb;
  const int g_begin = rb * gpb, g_end = min(ngroups, g_begin + gpb);
  // the next groups' A rows are fetched before this group's stores are issued (vmcnt
  // counts loads and stores in order: a load issued after the stores would wait for them)
  // FOLD: the folded value's raw x at this lane's output positions (row, 4 channels per
  // fragment), fetched with the group's A rows
  const T* X = (const T*)g.fx.x;
  // Range-checked loads over the block's rows (buf_ld16): a group past the block's range, a row
  // past M and k past K read zeros, with no branch and no select -- and the SE gate values of
  // the group come with its A rows (a gate load at the use waited for every load in flight).
  const auto rs_a = buf_rsrc(A + (size_t)g_begin * 16 * g.lda,
                             (long)(min(g_end * 16, M) - g_begin * 16) * g.lda * (long)sizeof(T));
  // (the SE-gated form for KS <= 2 only: its per-group gate vectors cost 16 KS registers; the
  // host routes a gated A with a deeper K elsewhere)
  constexpr bool GT = LAZY && KS <= 2;
  const bool has_gate = GT && g.lz.gate != nullptr;
  const auto rs_g = buf_rsrc(GT ? g.lz.gate : nullptr, has_gate ? (long)g.pyr.batch * K * 4 : 0);
  constexpr int NG = GT ? KS : 1;
  auto fetch = [&](int grp, uint4* v, float4 (*gv)[2], uint2* xv) {
    const int rl = (grp - g_begin) * 16 + (lane & 15), row = grp * 16 + (lane & 15);
    const bool gok = grp < g_end;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 32 * ks + kq;
      const uint32_t off = buf_off(k < K && gok, (uint32_t)((rl * g.lda + k) * (int)sizeof(T)));
      v[ks] = buf_ld16(rs_a, off);
      if constexpr (GT) {
        const uint32_t go = buf_off(k < K && gok && row < M, (uint32_t)(((row / hw) * K + k) * 4));
        gv[ks][0] = __builtin_bit_cast(float4, buf_ld16(rs_g, go));
        gv[ks][1] = __builtin_bit_cast(float4, buf_ld16(rs_g, go + 16));
      }
    }
    if constexpr (FOLD) {
#pragma unroll
      for (int f = 0; f < NF; ++f) {
        const int n0 = 16 * f + 4 * (lane >> 4);
        const bool ok = n0 < N && grp < g_end && row < M;
        const uint2 t = *reinterpret_cast<const uint2*>(X + (ok ? (size_t)row * g.fx.ld + nb0 + n0 : 0));
        xv[f] = ok ? t : make_uint2(0, 0);
      }
    }
  };
  // one 16-row group: transform + MFMA into the wave's staging rows, the refill of this slot
  // (GS_PF groups ahead) issued before the group's stores (vmcnt counts loads and stores in
  // order: a load issued after the stores would wait for them), then the stores.  Slots are
  // compile-time (the loop below is unrolled by GS_PF): rotating in-flight registers through a
  // rolled loop made the compiler wait for each load where its register was moved.
  auto group = [&](int grp, uint4 (&pre)[KS], float4 (&pg)[NG][2], uint2 (&prex)[FOLD ? NF : 1]) {
    const int row = grp * 16 + (lane & 15);
    if (g.has_stats && grp * 16 >= seg_end) {  // wave-uniform; segments start on 128-row multiples
      int send;
      const int sg = seg_of_row_end(g.pyr, grp * 16, send);  // (padding rows past a segment map to it)
      if (sg != cur_seg) {
        if (cur_seg >= 0) wflush(cur_seg);
        cur_seg = sg;
        seg_end = send;
      }
    }
    const bool live = row < M && row < seg_end;
    bf16x8_t bfrag[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      uint4 rv = pre[ks];
      if constexpr (LAZY) {
        const int k0 = 32 * ks + kq;
        float x[8];
        const uint32_t w4[4] = {rv.x, rv.y, rv.z, rv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          x[2 * i] = __uint_as_float(w4[i] << 16);
          x[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
        }
        const int kg = GT ? ks : 0;
        const float gt[8] = {pg[kg][0].x, pg[kg][0].y, pg[kg][0].z, pg[kg][0].w,
                             pg[kg][1].x, pg[kg][1].y, pg[kg][1].z, pg[kg][1].w};
        uint16_t o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float2 a = AFR ? af[AFR ? ks : 0][j] : af_s[32 * ks + kq + j];
          float u = x[j] * a.x + a.y;
          if constexpr (ACT == 1) u = swishf_(u);
          if (has_gate) u *= gt[j];
          o[j] = k0 + j < K ? f2bf(u) : (uint16_t)0;
        }
        rv = *reinterpret_cast<uint4*>(o);
      }
      bfrag[ks] = __builtin_bit_cast(bf16x8_t, rv);
    }
    uint2 xcur[FOLD ? NF : 1];
#pragma unroll
    for (int f = 0; f < (FOLD ? NF : 1); ++f) xcur[f] = prex[f];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      floatx4 d = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks][f], bfrag[ks], d, 0, 0, 0);
      const int n0 = 16 * f + 4 * (lane >> 4);
      const float4 bv = *reinterpret_cast<const float4*>(&bias_s[n0]);
      const float bias4[4] = {bv.x, bv.y, bv.z, bv.w};
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = d[r] + bias4[r];
        if constexpr (FOLD) {
          const float xf_ = __uint_as_float(r & 1 ? ((r < 2 ? xcur[f].x : xcur[f].y) & 0xffff0000u)
                                                  : ((r < 2 ? xcur[f].x : xcur[f].y) << 16));
          float du, dux;
          fold_terms(bf2f(f2bf(v[r])), xf_, ftab[n0 + r], g.fx.act, du, dux);
          if (live && n0 + r < N) { ss[f][r] += du; sq[f][r] += dux; }
        } else if (live) {
          ss[f][r] += v[r];
          sq[f][r] += v[r] * v[r];
        }
      }
      *reinterpret_cast<uint2*>(cw + (lane & 15) * LDW + n0) =
          make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16), (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
    }
    fetch(grp + GS_PF * 4, pre, pg, prex);
    // the 16 x N tile leaves as 16-byte vectors, a whole row range per store instruction
    // (a fixed number of store slots per lane, so the wait counts stay exact)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int vpr = N / 8, row0 = grp * 16;
#pragma unroll
    for (int i = 0; i < (32 * NF + 63) / 64; ++i) {
      const int e = lane + 64 * i;
      const int rl = e / vpr, c8 = (e - rl * vpr) * 8;
      if (e < 16 * vpr && row0 + rl < M)
        *reinterpret_cast<uint4*>(Y + (size_t)(row0 + rl) * g.ldc + nb0 + c8) = *reinterpret_cast<const uint4*>(cw + rl * LDW + c8);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  uint4 pre[GS_PF][KS];
  float4 pg[GS_PF][NG][2];
  uint2 prex[GS_PF][FOLD ? NF : 1];
#pragma unroll
  for (int u = 0; u < GS_PF; ++u) fetch(g_begin + wave + u * 4, pre[u], pg[u], prex[u]);
  for (int grp0 = g_begin + wave; grp0 < g_end; grp0 += 4 * GS_PF) {
#pragma unroll
    for (int u = 0; u < GS_PF; ++u) {
      if (grp0 + 4 * u >= g_end) break;
      group(grp0 + 4 * u, pre[u], pg[u], prex[u]);
    }
  }
  if (!g.has_stats) return;  // block-uniform
  if (cur_seg >= 0) wflush(cur_seg);
  __syncthreads();
  if (g_begin >= g_end) return;
  const int s_lo = seg_of_row(g.pyr, g_begin * 16), s_hi = seg_of_row(g.pyr, (g_end - 1) * 16);
  for (int sg = s_lo; sg <= s_hi; ++sg)
    for (int n = threadIdx.x; n < N; n += 256) {
      const float a = (red[sg][0][0][n] + red[sg][0][1][n]) + (red[sg][0][2][n] + red[sg][0][3][n]);
      const float b = (red[sg][1][0][n] + red[sg][1][1][n]) + (red[sg][1][2][n] + red[sg][1][3][n]);
      stat_put(g.stats.sum[sg], nb0 + n, (double)a);
      stat_put(g.stats.sq[sg], nb0 + n, (double)b);
    }
}

template <typename T, bool LAZY, int NF, int KS, bool FOLD = false>
static int launch_gemm_s(const GemmArgs& g, hipStream_t s) {
  const int ngroups = (g.M + 15) / 16;
  // 512 blocks (2 per CU): measured best over 512..2048 in the D0 step; 256 for the BiFPN /
  // head 64 -> 64 convs with statistics (fewer blocks flushing the same channels: 32768 rows
  // 17.4 -> 12.1 us), 1024 over 2M rows (2M x 32 -> 16: 50.1 -> 41.9 us) (scripts/kbench.py)
  int cap = 512;
  if (g.has_stats && g.N <= 64 && g.K >= 64 && g.M <= 262144) cap = 256;
  else if (g.M >= (1 << 21)) cap = 1024;
  if (dev_knob(7) > 0) cap = dev_knob(7);
  if (g.ncs > 1 && dev_knob(61) > 0) cap = dev_knob(61);
  const int ncs = g.ncs > 1 ? g.ncs : 1;
  const int grid = std::max(1, std::min(cdiv(ngroups, 4), std::max(1, cap / ncs))) * ncs;
  if constexpr (LAZY) {
    if (g.lz.act) EDET_LAUNCH((k_gemm_s<T, NF, KS, LAZY, FOLD, 1>), dim3(grid), dim3(256), 0, s, g);
    else EDET_LAUNCH((k_gemm_s<T, NF, KS, LAZY, FOLD, 0>), dim3(grid), dim3(256), 0, s, g);
  } else {
    EDET_LAUNCH((k_gemm_s<T, NF, KS, LAZY, FOLD, 0>), dim3(grid), dim3(256), 0, s, g);
  }
  return check_launch("edet gemm_s");
}

template <typename T, bool LAZY, int KS>
static int launch_gemm_s_n(const GemmArgs& g, hipStream_t s) {
  switch ((g.N + 15) / 16) {
    case 1: return launch_gemm_s<T, LAZY, 1, KS>(g, s);
    case 2: return launch_gemm_s<T, LAZY, 2, KS>(g, s);
    case 3: return launch_gemm_s<T, LAZY, 3, KS>(g, s);
    case 4: return launch_gemm_s<T, LAZY, 4, KS>(g, s);
    case 5: return launch_gemm_s<T, LAZY, 5, KS>(g, s);
    case 6: return launch_gemm_s<T, LAZY, 6, KS>(g, s);
    case 7: return launch_gemm_s<T, LAZY, 7, KS>(g, s);
    case 8: return launch_gemm_s<T, LAZY, 8, KS>(g, s);
    case 9: return launch_gemm_s<T, LAZY, 9, KS>(g, s);
    default: return launch_gemm_s<T, LAZY, 10, KS>(g, s);
  }
}

template <typename T, bool LAZY, int KS, bool FOLD = false>
static int launch_gemm_s_nf(const GemmArgs& g, int nf, hipStream_t s) {  // N <= 48
  if (nf <= 1) return launch_gemm_s<T, LAZY, 1, KS, FOLD>(g, s);
  if (nf == 2) return launch_gemm_s<T, LAZY, 2, KS, FOLD>(g, s);
  return launch_gemm_s<T, LAZY, 3, KS, FOLD>(g, s);
}

// K <= 32 and N <= 160 (a lazy A on one segment), and 32 < K <= 64, N <= 96 for a plain A
// (the 1x1 dgrads and the BiFPN / head pointwise convs), with BN statistics per segment on
// pyramids: rows between segments are padding, only ever written
template <typename T, bool LAZY>
static int dispatch_gemm_s(const GemmArgs& g, hipStream_t s, bool& done) {
  done = false;
  if (sizeof(T) != 2 || g.K % 8 || g.N % 8 || g.accumulate || g.ldc % 8 || g.lda % 8 || g.ldb % 8) return EDET_OK;
  // a plain A may span a pyramid (statistics per segment); the lazy transform reads segment
  // 0's BN affine and SE gate
  if (g.K <= 32 && g.N <= 160 && (g.pyr.nseg == 1 || !LAZY)) {
    done = true;
    return launch_gemm_s_n<T, LAZY, 1>(g, s);
  }
  // a lazy A up to K = 64 into N <= 64 on one segment (131072 x 40 -> 64 with BN + swish: 43 ->
  // 25 us; route sweep r03y)
  if (LAZY && g.K <= 64 && g.N <= 64 && g.pyr.nseg == 1) {
    done = true;
    return launch_gemm_s_n<T, LAZY, 2>(g, s);
  }
  if (!LAZY && g.K <= 64 && g.N <= 96) {
    done = true;
    return launch_gemm_s_n<T, LAZY, 2>(g, s);
  }
  // narrow outputs (N <= 48) over a deeper plain A (K <= 256): 2M x 96 -> 16 dgrad 259 -> 94 us,
  // 524288 x 144 -> 24 fwd 97 -> 33 us, dgrad 84 -> 29 us, 131072 x 240 -> 40 fwd 33 -> 24 us
  // (kbench r03w / r03x: conv1x1 4.86 -> 4.45 ms per step; the A-resident form staged the A tile
  // through LDS for a 16- to 40-column product).  Development slot 23 = 2: off
  if constexpr (!LAZY && sizeof(T) == 2) {
    if (dev_knob(23) != 2 && g.K <= 256 && g.N <= 48) {
      done = true;
      const int nf = cdiv(g.N, 16);
      switch (cdiv(g.K, 32)) {
        case 3: return launch_gemm_s_nf<T, LAZY, 3>(g, nf, s);
        case 4: return launch_gemm_s_nf<T, LAZY, 4>(g, nf, s);
        case 5: return launch_gemm_s_nf<T, LAZY, 5>(g, nf, s);
        case 6: return launch_gemm_s_nf<T, LAZY, 6>(g, nf, s);
        case 7: return launch_gemm_s_nf<T, LAZY, 7>(g, nf, s);
        default: return launch_gemm_s_nf<T, LAZY, 8>(g, nf, s);
      }
    }
  }
  return EDET_OK;
}

// Column-sliced wave streaming for the wide expand convs (K <= 192 into N > 160: 32768 x 112 ->
// 672, 8192 x 192 -> 1152, 131072 x 40 -> 240, 32768 x 80 -> 480).  The K-loop tiles ran these
// write-heavy products at 0.9-1.8 TB/s: each 64 x 128 tile block lived through a short K loop
// and its own epilogue, one round trip after another.  Here a wave keeps 16 NF columns of W in
// registers and streams its row groups (the A rows are re-read per slice, from L2).
// Development slot 59: 1 = wherever it applies, 2 = never; slot 60: NF; slot 61: blocks.
template <typename T, bool LAZY>
static int dispatch_gemm_s_sliced(GemmArgs g, hipStream_t s, bool& done) {
  done = false;
  const int route = dev_knob(59);
  if (route == 2 || sizeof(T) != 2) return EDET_OK;
  if (g.K % 8 || g.N % 8 || g.accumulate || g.ldc % 8 || g.lda % 8 || g.ldb % 8 || g.K > 192 || g.N <= 160)
    return EDET_OK;
  if (LAZY && (g.pyr.nseg != 1 || (g.lz.gate != nullptr && g.K > 64))) return EDET_OK;
  // Not a production route: in isolated replays a lazy A with K <= 128 over >= 32768 rows gained
  // (kbench r06q / r06r: 131072 x 40 -> 240 43.0 -> 35.5 us, 32768 x 112 -> 672 36.8 -> 33.6,
  // 32768 x 80 -> 480 24.7 -> 23.5; the 8192-row K = 192 expand lost, 24.1 -> 37.6), but the
  // same-box whole-step A/B did not move (12.074 vs 12.073 ms, profiles/r06/r06r_*): kept
  // behind slot 59 for the next study of these write-heavy products
  if (route != 1) return EDET_OK;
  const int KS = cdiv(g.K, 32);
  const int nf = dev_knob(60) > 0 ? dev_knob(60) : (KS <= 4 ? 4 : 2);
  g.ncs = cdiv(g.N, 16 * nf);
  done = true;
  auto go = [&](auto ks_c) -> int {
    constexpr int KSC = decltype(ks_c)::value;
    return nf == 2 ? launch_gemm_s<T, LAZY, 2, KSC>(g, s) : launch_gemm_s<T, LAZY, 4, KSC>(g, s);
  };
  switch (KS) {
    case 1: return go(std::integral_constant<int, 1>{});
    case 2: return go(std::integral_constant<int, 2>{});
    case 3: return go(std::integral_constant<int, 3>{});
    case 4: return go(std::integral_constant<int, 4>{});
    case 5: return go(std::integral_constant<int, 5>{});
    default: return go(std::integral_constant<int, 6>{});
  }
}

// ------------------------------------------------------------------ launch helpers
template <typename T, int BM, int BN, bool LAZY, int KC = 32, int FOLD = 0>
static int launch_gemm(GemmArgs g, hipStream_t s) {
  // accumulating launches (the plain dgrads of multi-consumer values) take the ACC instance
  if constexpr (!LAZY && FOLD == 0) {
    if (g.accumulate) {
      g.ntm = cdiv(g.M, BM);
      g.ntn = cdiv(g.N, BN);
      const int nwg = g.ntm * g.ntn;
      if (nwg == 0) return EDET_OK;
      EDET_LAUNCH((k_gemm<T, BM, BN, KC, false, 0, true>), dim3(nwg), dim3(256), 0, s, g);
      return check_launch("edet gemm (accumulate)");
    }
  }
  g.ntm = cdiv(g.M, BM);
  g.ntn = cdiv(g.N, BN);
  const int nwg = g.ntm * g.ntn;
  if (nwg == 0) return EDET_OK;
  const int nimg = (LAZY && g.lz.gate) ? gemm_gate_imgs(BM, g.pyr.H[0] * g.pyr.W[0], g.pyr.batch) : 0;
  const size_t dyn = LAZY ? (size_t)g.K * (sizeof(float2) + nimg * sizeof(float)) : 0;
  EDET_LAUNCH((k_gemm<T, BM, BN, KC, LAZY, FOLD>), dim3(nwg), dim3(256), dyn, s, g);
  return check_launch("edet gemm");
}

// gemm_r's LDS image; nimg = SE gate rows staged per tile (gemm_gate_imgs, 0 without a gate)
template <typename T, int BM, bool LAZY>
static size_t gemm_r_lds(int K, int KP, int LDC, int nimg = 2) {
  return (size_t)(BM + (KP <= 128 ? 2 : 1) * RNB) * (KP + 8) * sizeof(T) + (size_t)BM * LDC * sizeof(T) +
         5 * (size_t)LDC * sizeof(float) +
         (LAZY ? (size_t)K * (sizeof(float2) + nimg * sizeof(float)) : 0);
}

template <typename T, int BM, bool LAZY>
static int launch_gemm_r(GemmArgs g, hipStream_t s) {
  const int KP = cdiv(g.K, 32) * 32;
  const int ntm = cdiv(g.M, BM);
  const int nch = cdiv(g.N, RNB);
  int nsplit = 1;
  while (nsplit < nch && (long)ntm * nsplit < 1024) nsplit *= 2;
  if (nsplit > nch) nsplit = nch;
  int cps = cdiv(nch, nsplit);
  // narrow the per-block column range until the staged C tile fits
  const int nimg = (LAZY && g.lz.gate) ? gemm_gate_imgs(BM, g.pyr.H[0] * g.pyr.W[0], g.pyr.batch) : 0;
  while (cps > 1 && gemm_r_lds<T, BM, LAZY>(g.K, KP, cps * RNB, nimg) > 150 * 1024) cps = cdiv(cps, 2);
  nsplit = cdiv(nch, cps);
  const int LDC = nsplit == 1 ? cdiv(g.N, 8) * 8 : cps * RNB;
  const size_t lds = gemm_r_lds<T, BM, LAZY>(g.K, KP, LDC, nimg);
  EDET_REQUIRE(lds <= 160 * 1024, "edet gemm_r: tile does not fit LDS (K=%d N=%d)", g.K, g.N);
  if (ntm == 0) return EDET_OK;
  // resident blocks per CU from the LDS image; the row-tile workers per split fill that once
  const int per_cu = max(1, min(8, (int)((160 * 1024) / lds)));
  const int G = min(ntm, max(1, cdiv(256 * per_cu, nsplit)));
  // in-place B chunk loads batched (stage_rows) for K > 128: D4 (K = 224 BiFPN / head convs)
  // conv1x1 19.5 -> 18.9 ms per step in kbench, D0 even (r03r); development slot 24 = 2: cp8 loop
  const int bstage = dev_knob(24) != 2;
  EDET_LAUNCH((k_gemm_r<T, BM, LAZY>), dim3(G * nsplit), dim3(256), lds, s, g, KP, nsplit, cps, LDC, bstage);
  return check_launch("edet gemm_r");
}

// K > 512 with one full-N tile (N <= 320): streaming K loop
template <typename T, bool LAZY, int FOLD = 0>
static int dispatch_gemm_kloop(GemmArgs g, hipStream_t s) {
  const int NP = cdiv(g.N, 32) * 32;
  // BM = 32 when 64-row tiles would leave the chip under-filled (and for the fp32 fold, whose
  // staged C and x tiles at 64 x 320 would not fit the LDS)
  constexpr bool only32 = FOLD != 0 && sizeof(T) == 4;
#ifdef EDET_DEV
  // development slots 42 / 43: force the row / column tile (32, 64, 128 / 64, 128, 256)
  if constexpr (!only32 && FOLD == 0) {
    if (const int bm = dev_knob(42)) {
      const int bn = dev_knob(43) ? dev_knob(43) : (NP <= 64 ? 64 : 128);
      if (bm == 128 && bn == 64) return launch_gemm<T, 128, 64, LAZY, 32, FOLD>(g, s);
      if (bm == 128 && bn == 128) return launch_gemm<T, 128, 128, LAZY, 32, FOLD>(g, s);
      if (bm == 64 && bn == 64) return launch_gemm<T, 64, 64, LAZY, 32, FOLD>(g, s);
      if (bm == 64 && bn == 128) return launch_gemm<T, 64, 128, LAZY, 32, FOLD>(g, s);
      if (bm == 64 && bn == 256) return launch_gemm<T, 64, 256, LAZY, 32, FOLD>(g, s);
      if (bm == 32 && bn == 64) return launch_gemm<T, 32, 64, LAZY, 32, FOLD>(g, s);
      if (bm == 32 && bn == 128) return launch_gemm<T, 32, 128, LAZY, 32, FOLD>(g, s);
      if (bm == 32 && bn == 256) return launch_gemm<T, 32, 256, LAZY, 32, FOLD>(g, s);
    }
  }
#endif
  // Round-6 tile sweep of the plain, statistics-free products (the 1x1 dgrads; development slots
  // 42 / 43, profiles/r06/r06ap_gemm_tile_sweep.txt): a short K loop into a wide output wants
  // column tiles -- more blocks, A re-read per tile from L2 -- (131072 x 40 -> 240: 33.5 -> 22.3
  // us, 32768 x 80 -> 240: 12.9 -> 10.3), and the class head's deep dgrad 128-row tiles
  // (174592 x 729 -> 64: 66.0 -> 59.5)
  if constexpr (FOLD == 0 && !LAZY && sizeof(T) == 2) {
    if (!g.has_stats && g.M >= 131072 && g.K <= 64 && NP > 64) return launch_gemm<T, 64, 64, LAZY, 32, FOLD>(g, s);
    if (!g.has_stats && g.M >= 131072 && g.K > 512 && NP <= 64) return launch_gemm<T, 128, 64, LAZY, 32, FOLD>(g, s);
    if (!g.has_stats && g.M >= 32768 && g.M < 131072 && g.K <= 128 && NP > 128 && NP <= 320)
      return launch_gemm<T, 64, 128, LAZY, 32, FOLD>(g, s);
  }
  if (only32 || cdiv(g.M, 64) < 512) {
    if (NP <= 64) return launch_gemm<T, 32, 64, LAZY, 32, FOLD>(g, s);
    if (NP <= 96) return launch_gemm<T, 32, 96, LAZY, 32, FOLD>(g, s);
    if (NP <= 128) return launch_gemm<T, 32, 128, LAZY, 32, FOLD>(g, s);
    if (NP <= 192) return launch_gemm<T, 32, 192, LAZY, 32, FOLD>(g, s);
    if (NP <= 320) return launch_gemm<T, 32, 320, LAZY, 32, FOLD>(g, s);
  } else if constexpr (!only32) {
    if (NP <= 64) return launch_gemm<T, 64, 64, LAZY, 32, FOLD>(g, s);
    if (NP <= 96) return launch_gemm<T, 64, 96, LAZY, 32, FOLD>(g, s);
    if (NP <= 128) return launch_gemm<T, 64, 128, LAZY, 32, FOLD>(g, s);
    if (NP <= 192) return launch_gemm<T, 64, 192, LAZY, 32, FOLD>(g, s);
    if (NP <= 320) return launch_gemm<T, 64, 320, LAZY, 32, FOLD>(g, s);
  }
  // wider outputs (EfficientDet-D4+ project convs: K = 1632 -> N = 448): 128-column tiles
  // (r03p sweep: 64-deep K chunks, 256-column tiles or both were 1.15-1.8x slower)
  if constexpr (!only32)
    if (cdiv(g.M, 64) >= 512) return launch_gemm<T, 64, 128, LAZY, 32, FOLD>(g, s);
  return launch_gemm<T, 32, 128, LAZY, 32, FOLD>(g, s);
}

// dgrad with the BN-backward fold of the gradient's value (plain A, no statistics): the
// wave-streaming form where it applies to one segment, else the K loop (any shape, pyramids)
template <typename T>
static int dispatch_dgrad_fold(const GemmArgs& g, hipStream_t s) {
  if constexpr (sizeof(T) == 2) {
    const bool vec = g.K % 8 == 0 && g.N % 8 == 0 && g.ldc % 8 == 0 && g.lda % 8 == 0 && g.ldb % 8 == 0 &&
                     g.fx.ld % 8 == 0 && !g.accumulate && g.pyr.nseg == 1;
    if (vec && g.K <= 64 && g.N <= 96) {
      switch (cdiv(g.N, 16)) {
        case 1: return launch_gemm_s<T, false, 1, 2, true>(g, s);
        case 2: return launch_gemm_s<T, false, 2, 2, true>(g, s);
        case 3: return launch_gemm_s<T, false, 3, 2, true>(g, s);
        case 4: return launch_gemm_s<T, false, 4, 2, true>(g, s);
        case 5: return launch_gemm_s<T, false, 5, 2, true>(g, s);
        default: return launch_gemm_s<T, false, 6, 2, true>(g, s);
      }
    }
    if (vec && g.K <= 256 && g.N <= 48) {
      const int nf = cdiv(g.N, 16);
      switch (cdiv(g.K, 32)) {
        case 3: return launch_gemm_s_nf<T, false, 3, true>(g, nf, s);
        case 4: return launch_gemm_s_nf<T, false, 4, true>(g, nf, s);
        case 5: return launch_gemm_s_nf<T, false, 5, true>(g, nf, s);
        case 6: return launch_gemm_s_nf<T, false, 6, true>(g, nf, s);
        case 7: return launch_gemm_s_nf<T, false, 7, true>(g, nf, s);
        default: return launch_gemm_s_nf<T, false, 8, true>(g, nf, s);
      }
    }
  }
  return dispatch_gemm_kloop<T, false, true>(g, s);
}

template <typename T, bool LAZY>
static int dispatch_gemm(GemmArgs g, hipStream_t s) {
  auto gemm_r_imgs = [&](int bm) {  // SE gate rows gemm_r stages per tile
    return (LAZY && g.lz.gate) ? gemm_gate_imgs(bm, g.pyr.H[0] * g.pyr.W[0], g.pyr.batch) : 0;
  };
  const int KP0 = cdiv(g.K, 32) * 32;
#ifdef EDET_DEV
  // development slot 26: force a kernel family where it applies (1 = wave-streaming, 2 =
  // B-resident, 3 = A-resident, 4 = K loop) for route sweeps; otherwise the production rules
  if (const int route = dev_knob(26)) {
    const int KP = cdiv(g.K, 32) * 32, LDCf = cdiv(g.N, 8) * 8;
    if (route == 1 && sizeof(T) == 2 && g.K % 8 == 0 && g.N % 8 == 0 && !g.accumulate && g.ldc % 8 == 0 &&
        g.lda % 8 == 0 && g.ldb % 8 == 0 && g.K <= 256 && g.N <= 160 && (!LAZY || g.pyr.nseg == 1)) {
      switch (cdiv(g.K, 32)) {
        case 1: return launch_gemm_s_n<T, LAZY, 1>(g, s);
        case 2: return launch_gemm_s_n<T, LAZY, 2>(g, s);
        case 3: return launch_gemm_s_n<T, LAZY, 3>(g, s);
        case 4: return launch_gemm_s_n<T, LAZY, 4>(g, s);
        case 5: return launch_gemm_s_n<T, LAZY, 5>(g, s);
        case 6: return launch_gemm_s_n<T, LAZY, 6>(g, s);
        case 7: return launch_gemm_s_n<T, LAZY, 7>(g, s);
        default: return launch_gemm_s_n<T, LAZY, 8>(g, s);
      }
    }
    if (route == 2 && g.ldc % 8 == 0 && g.lda % 8 == 0 && g.K % 8 == 0 && g.M > 0) {
      PwPlan p;
      int FN;
      bool ks;
      if (pw_plan(g, LAZY, sizeof(T), p, FN, ks)) {
        if (!ks) return launch_pwb<T, 2, false, LAZY>(g, p, s);
        if (FN == 2) return launch_pwb<T, 2, true, LAZY>(g, p, s);
        return launch_pwb<T, 1, true, LAZY>(g, p, s);
      }
    }
    if (route == 3 && g.K <= 512) {
      if (gemm_r_lds<T, 128, LAZY>(g.K, KP, LDCf, gemm_r_imgs(128)) <= 96 * 1024) return launch_gemm_r<T, 128, LAZY>(g, s);
      if (gemm_r_lds<T, 64, LAZY>(g.K, KP, LDCf, gemm_r_imgs(64)) <= 96 * 1024) return launch_gemm_r<T, 64, LAZY>(g, s);
      if (gemm_r_lds<T, 32, LAZY>(g.K, KP, LDCf, gemm_r_imgs(32)) <= 96 * 1024) return launch_gemm_r<T, 32, LAZY>(g, s);
    }
    if (route == 4) return dispatch_gemm_kloop<T, LAZY>(g, s);
  }
#endif
  // Round-4 route sweep (development slot 26 over every D0 and D4 conv1x1 launch after the
  // loaders were made countable, profiles/r04ad_route_sweep/): the K loop now wins the plain,
  // statistics-free K = 224 products into N >= 192 (the D4 head / BiFPN dgrads and the class
  // predict: 174592 x 224 -> 224 dgrad 87 -> 67 us, -> 729 fwd 254 -> 200 us) and a lazy A
  // with K > 64 into 192 < N <= 320 (D4 32768 x 160 -> 224: 95 -> 59 us); the A-resident form
  // wins K = 224 into N >= 192 with statistics at M <= 8192 (8192 x 224 -> 224: 33 -> 24 us);
  // the B-resident form wins the D0 class predict (174592 x 64 -> 729: 114 -> 93 us)
  {
    bool done = false;
    const int rc = dispatch_gemm_s_sliced<T, LAZY>(g, s, done);
    if (done || rc) return rc;
  }
  if constexpr (sizeof(T) == 2) {
    // Round-5 K-loop tile sweep over the mid-size D0 products (8192 / 32768 rows: the 16^2 and
    // 32^2 stages, 0.4-1.6 TB/s; tools/gpu_r05l.sh, profiles/r05/r05l_gemm_tiles.txt): 64-column
    // tiles with more rows per tile -- more blocks than the one full-N tile, and fewer blocks
    // per output column flushing BN statistics (one fp64 atomic per column per block)
    if (g.M >= 8192 && g.M <= 65536) {
      // plain A with statistics, deep K (the project convs): 8192 x 1152 -> 192 24.5 -> 16.0 us,
      // 32768 x 672 -> 112 26.7 -> 21.0
      if (!LAZY && g.has_stats && g.K > 256 && g.N <= 320)
        return g.M <= 16384 ? launch_gemm<T, 64, 64, LAZY>(g, s) : launch_gemm<T, 128, 64, LAZY>(g, s);
      // plain dgrads at 8192 rows: 8192 x 1152 -> 320 25.0 -> 20.1 us, 192 -> 1152 18.9 -> 13.9
      if (!LAZY && !g.has_stats && g.M <= 16384 && g.K >= 64 && g.N >= 64)
        return g.N <= 192 ? launch_gemm<T, 64, 64, LAZY>(g, s) : launch_gemm<T, 128, 64, LAZY>(g, s);
      // lazy A into wide outputs at 8192 rows (the stage-6 expand convs): 29.5 -> 25.7 us
      if (LAZY && g.M <= 16384 && g.K > 64 && g.N > 320) return launch_gemm<T, 64, 128, LAZY>(g, s);
      // lazy A with statistics into 64 columns (the BiFPN input projections): 17.4 -> 13.8 us
      if (LAZY && g.has_stats && g.K > 64 && g.N <= 64 && g.M <= 32768)
        return g.M <= 8192 ? launch_gemm<T, 64, 64, LAZY>(g, s) : launch_gemm<T, 128, 64, LAZY>(g, s);
    }
    const int KPr = cdiv(g.K, 32) * 32;
    const bool w224 = g.N >= 192 && KPr > 192 && KPr <= 224;
    if (!LAZY && !g.has_stats && w224) return dispatch_gemm_kloop<T, LAZY>(g, s);
    if (LAZY && g.K > 64 && g.N > 192 && g.N <= 320) return dispatch_gemm_kloop<T, LAZY>(g, s);
    if (!LAZY && g.has_stats && w224 && g.M <= 8192 && g.K <= 512) {
      const int LDCf = cdiv(g.N, 8) * 8;
      if (gemm_r_lds<T, 32, LAZY>(g.K, KPr, LDCf, 0) <= 96 * 1024) return launch_gemm_r<T, 32, LAZY>(g, s);
    }
    if (!LAZY && !g.has_stats && g.K <= 64 && g.N > 640 && g.M >= 131072) {
      bool done = false;
      const int rc = dispatch_pwb_forced<T, LAZY>(g, s, done);
      if (done || rc) return rc;
    }
  }
  {
    bool done = false;
    const int rc = dispatch_gemm_s<T, LAZY>(g, s, done);
    if (done || rc) return rc;
  }
  // route sweep over every D0 conv1x1 launch (r03y, development slot 26): past the
  // wave-streaming shapes, the pipelined K loop beats the B- and A-resident forms for a plain A
  // without BN statistics (the 1x1 dgrads and the box predict: 32768 x 112 -> 672 dgrad 93 -> 47
  // us, 174592 x 64 -> 36 38 -> 14 us; about -150 us per step), and for a lazy A with K > 64 into
  // N > 320 (32768 x 80 -> 480: 106 -> 87 us).  D4's K = 224 convs stay B-resident (below).
  const bool wide224 = g.N >= 192 && KP0 > 192 && KP0 <= 224;
  if ((!LAZY && !g.has_stats && !wide224) || (LAZY && g.K > 64 && g.N > 320)) return dispatch_gemm_kloop<T, LAZY>(g, s);
  {
    bool done = false;
    const int rc = dispatch_pwb<T, LAZY>(g, s, done);
    if (done || rc) return rc;
  }
  // A-resident kernel whenever its LDS image fits (<= 96 KB: >= 1 block per CU with room);
  // BM = rows per block chosen as the largest that fits.  Otherwise stream K (N <= 320).
  const int KP = cdiv(g.K, 32) * 32;
  const int LDCf = cdiv(g.N, 8) * 8;
  constexpr size_t BUDGET = 96 * 1024;
  // (lazy A with K > 64 into N > 320 took the K loop above: the A-resident form walks its
  // column chunks one dependent B load at a time with 2 blocks per CU; 8192x192x1152,
  // 32768x112x672 measured 1.3-1.4x faster on the K loop)
  if (g.K <= 512) {
    // the largest row tile that still gives >= 256 (row tile, column chunk) blocks: at M = 8192
    // the 128-row tiles left 64 blocks for 256 CUs (8192 x 320 -> 64: 21 us)
    const bool fills = (long)cdiv(g.M, 128) * cdiv(g.N, RNB) >= 256;  // (21 -> 19 us at 8192 x 320 -> 64)
    if (!fills && gemm_r_lds<T, 32, LAZY>(g.K, KP, LDCf, gemm_r_imgs(32)) <= BUDGET) return launch_gemm_r<T, 32, LAZY>(g, s);
    if (gemm_r_lds<T, 128, LAZY>(g.K, KP, LDCf, gemm_r_imgs(128)) <= BUDGET) return launch_gemm_r<T, 128, LAZY>(g, s);
    if (gemm_r_lds<T, 64, LAZY>(g.K, KP, LDCf, gemm_r_imgs(64)) <= BUDGET) return launch_gemm_r<T, 64, LAZY>(g, s);
    if (gemm_r_lds<T, 32, LAZY>(g.K, KP, LDCf, gemm_r_imgs(32)) <= BUDGET) return launch_gemm_r<T, 32, LAZY>(g, s);
    // wider C tiles than fit: the column-split A-resident form walked its chunks one
    // dependent B load at a time with one block per CU (dgrad 8192 x 320 -> 1152: 88 us);
    // the pipelined K loop over 128-column tiles takes 31 us
  }
  return dispatch_gemm_kloop<T, LAZY>(g, s);
}

static bool lazy_is_plain(const edet_lazy* a) {
  return a->bn.enabled == 0 && a->act == EDET_ACT_NONE && a->gate == nullptr;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_conv1x1_fwd(int dtype, const edet_lazy* a, const edet_pyramid* rows, int K,
                     const void* wt, int N, const float* bias, void* y, int ldy,
                     int accumulate, const edet_statout* stats, edet_stream_t stream) {
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
  // the lazy K-loop instances store without reading C (the accumulating instance is the plain
  // dgrads' compile-time case): an accumulating forward needs a plain A
  EDET_REQUIRE(!accumulate || plain, "conv1x1_fwd: accumulate=1 needs a plain A (no BN / act / gate)");
  EDET_DTYPE_DISPATCH(dtype, T, {
    return plain ? dispatch_gemm<T, false>(g, s) : dispatch_gemm<T, true>(g, s);
  });
}

int edet_conv1x1_dgrad(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                       const void* wkn, int K, void* dx, int lddx, int accumulate,
                       edet_stream_t stream) {
  EDET_REQUIRE(dy && rows && wkn && dx, "conv1x1_dgrad: null argument");
  EDET_REQUIRE(lddy % 8 == 0 && K % 8 == 0 && N > 0, "conv1x1_dgrad: need lddy%%8==0, K%%8==0");
  GemmArgs g{};
  g.a = dy; g.b = wkn; g.c = dx; g.bias = nullptr; g.pyr = *rows;
  g.lda = lddy; g.ldb = cdiv(N, 8) * 8; g.ldc = lddx;
  g.M = pyr_total_rows(*rows); g.K = N; g.N = K;  // GEMM K = conv out channels
  g.accumulate = accumulate; g.has_stats = 0;
  hipStream_t s = (hipStream_t)stream;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_gemm<T, false>(g, s); });
}

int edet_conv1x1_dgrad_fold(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                            const void* wkn, int K, void* dx, int lddx, const edet_lazy* xv,
                            const edet_bngrad64* fold, edet_stream_t stream) {
  EDET_REQUIRE(dy && rows && wkn && dx && xv && xv->x && fold, "conv1x1_dgrad_fold: null argument");
  EDET_REQUIRE(lddy % 8 == 0 && K % 8 == 0 && N > 0 && lddx % 8 == 0 && xv->ld % 8 == 0,
               "conv1x1_dgrad_fold: need lddy, K, lddx, x->ld multiples of 8");
  EDET_REQUIRE(xv->bn.enabled && xv->gate == nullptr, "conv1x1_dgrad_fold: the folded value needs BN and no gate");
  EDET_REQUIRE(rows->nseg >= 1 && rows->nseg <= EDET_MAX_SEG, "conv1x1_dgrad_fold: bad pyramid");
  for (int i = 0; i < rows->nseg; ++i)
    EDET_REQUIRE(fold->dgamma[i] && fold->dbeta[i], "conv1x1_dgrad_fold: null fold destination (segment %d)", i);
  GemmArgs g{};
  g.a = dy; g.b = wkn; g.c = dx; g.bias = nullptr; g.pyr = *rows;
  g.lda = lddy; g.ldb = cdiv(N, 8) * 8; g.ldc = lddx;
  g.M = pyr_total_rows(*rows); g.K = N; g.N = K;  // GEMM K = conv out channels
  g.accumulate = 0;
  g.has_stats = 1;  // the statistics flush carries (sum du -> dbeta, sum du * xhat -> dgamma)
  for (int i = 0; i < rows->nseg; ++i) { g.stats.sum[i] = fold->dbeta[i]; g.stats.sq[i] = fold->dgamma[i]; }
  g.fx = *xv;
  hipStream_t s = (hipStream_t)stream;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_dgrad_fold<T>(g, s); });
}

int edet_conv1x1_dgrad_sesum(int dtype, const void* dy, int lddy, const edet_pyramid* rows, int N,
                             const void* wkn, int K, void* dx, int lddx, const edet_lazy* yv, double* sums5,
                             edet_stream_t stream) {
  EDET_REQUIRE(dy && rows && wkn && dx && yv && yv->x && sums5, "conv1x1_dgrad_sesum: null argument");
  EDET_REQUIRE(lddy % 8 == 0 && K % 8 == 0 && N > 0 && lddx % 8 == 0 && yv->ld % 8 == 0,
               "conv1x1_dgrad_sesum: need lddy, K, lddx, y->ld multiples of 8");
  EDET_REQUIRE(yv->bn.enabled && yv->act == EDET_ACT_SWISH && rows->nseg == 1 && K <= 2048,
               "conv1x1_dgrad_sesum: needs swish(bn(y)) on one segment, C <= 2048");
  const int B = rows->batch, HW = rows->H[0] * rows->W[0];
  edet_lazy y = *yv;
  y.gate = nullptr;  // the sums are of the pre-gate value's terms (k_gate_bn_reduce)
  // Route: the project dgrads the wave-streaming GEMM takes (GEMM K <= 32, N <= 160: the
  // stage 0-1 convs) and planes whose tiles could straddle images keep the separate pass
  const bool narrow = dtype == EDET_BF16 && N <= 32 && K <= 160;
  if (narrow || HW % 64 != 0 || rows->row_off[0] != 0) {
    int rc = edet_conv1x1_dgrad(dtype, dy, lddy, rows, N, wkn, K, dx, lddx, 0, stream);
    if (rc) return rc;
    return edet_gate_bn_reduce(dtype, &y, B, HW, K, dx, sums5, stream);
  }
  GemmArgs g{};
  g.a = dy; g.b = wkn; g.c = dx; g.bias = nullptr; g.pyr = *rows;
  g.lda = lddy; g.ldb = cdiv(N, 8) * 8; g.ldc = lddx;
  g.M = pyr_total_rows(*rows); g.K = N; g.N = K;  // GEMM K = conv out channels
  g.accumulate = 0;
  g.has_stats = 0;
  g.fx = y;
  g.se5 = sums5; g.se_batch = B;
  hipStream_t s = (hipStream_t)stream;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_gemm_kloop<T, false, 2>(g, s); });
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
  hipStream_t s = (hipStream_t)stream;
  const bool plain = lazy_is_plain(a);
  // narrow outputs over very long M (the stage 0-1 convs: 2M x 16 -> 96, 2M x 32 -> 16): every
  // wave streams its own rows against the whole N x K tile (k_wgs), each operand read once.
  // Wider tiles need too many accumulators for the occupancy this stream wants (measured
  // slower than the 64x64 cooperative tiles below on every other D0 shape, scripts/wg_probe.py)
  const bool wide = dev_knob(3) == 1;
  if (dtype == EDET_BF16 && plain && K % 8 == 0 &&
      (wide || (cdiv(N, 16) * cdiv(K, 16) <= 6 && g.M >= (1 << 18)))) {
    const WgsShape t = pick_wgs(N, K, wide);
    WgsArgs w{};
    w.a = (const uint16_t*)a->x; w.dy = (const uint16_t*)dy; w.dw = dwt; w.db = dbias; w.pyr = *rows;
    w.lda = a->ld; w.lddy = lddy; w.M = g.M; w.K = K; w.N = N;
    w.ntk = cdiv(cdiv(K, 16), t.fk);
    const int wtiles = cdiv(cdiv(N, 16), t.fn) * w.ntk;
    w.ngrp = cdiv(g.M, 32);
    // 512 blocks of 4 waves, at least 16 row groups per wave; the block's folded tile goes out
    // as fp32 atomics (N*K per block: 1.5K floats at 96 x 16)
    const int wblocks = dev_knob(4) > 0 ? dev_knob(4) : 512, wmin = dev_knob(5) > 0 ? dev_knob(5) : 64;
    int splits = std::max(1, std::min(cdiv(wblocks, wtiles), w.ngrp / wmin));
    w.gpb = cdiv(w.ngrp, splits);
    w.splits = cdiv(w.ngrp, w.gpb);
    // every block's folded tile lands on the same N*K addresses: hundreds of fp32 atomic adders
    // per address serialise at the memory side, plain partial stores + the spread sum pass
    // do not (2M x 16 -> 96: 130 -> 95 us, 2M x 32 -> 16: 57 -> 40 us)
    w.part = w.splits > 1 ? workspace_f32((size_t)w.splits * ((size_t)N * K + N)) : nullptr;
    int rc = dispatch_wgs(w, t.fn, t.fk, wtiles * w.splits, s);
    if (rc || !w.part) return rc;
    return sum_partials(w.part, w.splits, (long)N * K, dwt, s, N, dbias);  // dW and db, one launch
  }
  if (dtype == EDET_BF16) {
    // lazy A (BN / act / gate applied while staging): 64x64 tiles with transposing LDS reads.
    // Stages never straddle a segment: segments start on 128-row boundaries.  ~2048 blocks of
    // at least 8 stages each, fp32 atomics into dW.
    // ~2048 blocks of >= 8 stages; a single 64x64 tile over a long M (the head / BiFPN
    // pointwise convs) or a short M: 4096 of >= 4 (174592 x 64 -> 64: 23.8 -> 17.6 us,
    // 2048 x 320 -> 64: 10.6 -> 7.7); >= 16 stages for many tiles over M <= 32768 (32768 x 112
    // -> 672: 36.8 -> 32.1 us), the class predict (106 -> 100) and M >= 524288 (38 -> 35)
    // (profiles/r02b_wgrad_plan_sweep.txt)
    // The BiFPN 64 -> 64 convs (one tile, M <= 32768) want ~8192 blocks of >= 2 stages (512 x 64
    // -> 64: 23.5 -> 18.0 us per step, 2048: 47.5 -> 37.2, 32768: 74.7 -> 66.9); a few tiles over
    // M <= 8192 >= 4 stages (8192 x 320 -> 64: 33.9 -> 28.5) (profiles/r03ab_wgrad_plan_sweep.txt)
    int target = 2048, min_stages = 8;
    if (tiles == 1 && g.M <= 32768) target = 8192, min_stages = 2;
    else if (tiles == 1 || g.M <= 4096) target = 4096, min_stages = 4;
    else if (tiles <= 8 && g.M <= 8192) min_stages = 4;
    else if ((tiles >= 22 && g.M <= 32768) || (tiles >= 12 && g.M >= 131072) || g.M >= 524288) min_stages = 16;
    if (dev_knob(0) > 0) target = dev_knob(0);
    if (dev_knob(1) > 0) min_stages = dev_knob(1);
    int split = cdiv(target, tiles);
    const int max_split = std::max(1, cdiv(g.M, WT_BM * min_stages));
    if (split > max_split) split = max_split;
    g.rows_per = cdiv(cdiv(g.M, split), WT_BM) * WT_BM;
    split = std::max(1, cdiv(g.M, g.rows_per));
    // few output tiles split over many row ranges: the same per-address atomic contention as
    // k_wgs, partials + the sum pass instead (524288 x 24 -> 144: 71 -> 63 us, 131072 x 40 ->
    // 240: 37 -> 27 us); many tiles keep the atomics (class predict 105 vs 124 us with partials)
    const bool use_part = dev_knob(2) == 1 || (dev_knob(2) == 0 && tiles <= 4 && split >= 128);
    g.part = use_part && split > 1 ? workspace_f32((size_t)split * ((size_t)N * K + N)) : nullptr;
    // stage rows / stages in flight (development slot 21: 1 = 64/3, 2 = 64/4, 3 = 128/2, 4 = 128/3)
    const int form = dev_knob(21);
    // (whole PF-stage rounds per block: a block runs its stages in rounds of PF)
    const int bm = (form >= 3 ? 128 : 64) * (form == 1 || form == 4 ? 3 : form == 2 ? 4 : 2);
    if (g.rows_per % bm) {
      g.rows_per = cdiv(g.rows_per, bm) * bm;
      split = std::max(1, cdiv(g.M, g.rows_per));
      if (g.part) g.part = workspace_f32((size_t)split * ((size_t)N * K + N));
    }
    const dim3 grid(tiles * split);
#define EDET_WGT(BM_, PF_)                                                            \
  do {                                                                                \
    if (plain) EDET_LAUNCH((k_wgrad_tr<false, BM_, PF_>), grid, dim3(256), 0, s, g); \
    else if (a->act) EDET_LAUNCH((k_wgrad_tr<true, BM_, PF_, 1>), grid, dim3(256), 0, s, g); \
    else EDET_LAUNCH((k_wgrad_tr<true, BM_, PF_, 0>), grid, dim3(256), 0, s, g);     \
  } while (0)
    switch (form) {
      case 1: EDET_WGT(64, 3); break;
      case 2: EDET_WGT(64, 4); break;
      case 3: EDET_WGT(128, 2); break;
      case 4: EDET_WGT(128, 3); break;
      default: EDET_WGT(64, 2); break;
    }
#undef EDET_WGT
    int rc = check_launch("edet wgrad");
    if (rc || !g.part) return rc;
    return sum_partials(g.part, split, (long)N * K, dwt, s, N, dbias);  // dW and db, one launch
  }
  int split = cdiv(2048, tiles);
  const int max_split = cdiv(g.M, 32 * 4);  // at least 4 row-chunks per block
  if (split > max_split) split = max_split;
  if (split < 1) split = 1;
  g.rows_per = cdiv(cdiv(g.M, split), 32) * 32;
  split = cdiv(g.M, g.rows_per);
  if (split < 1) split = 1;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (plain) EDET_LAUNCH((k_wgrad<T, false>), dim3(tiles * split), dim3(256), 0, s, g);
    else EDET_LAUNCH((k_wgrad<T, true>), dim3(tiles * split), dim3(256), 0, s, g);
    return check_launch("edet wgrad");
  });
}

}  // extern "C"
