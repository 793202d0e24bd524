// Fused optimizer step over the flat fp32 parameter buffer:
//   g' = g + l2 * w            (efficientdet_net_train.py:21-28, 4e-5 * sum l2_loss(kernels))
//   gnorm = ||g'||_2; g' *= clip / max(gnorm, clip)   (tf.clip_by_global_norm, :129-130)
//   v = m v - lr g'; w += v                           (Keras SGD momentum, train.py:114-115)
//   ema -= (1 - d)(ema - w)                           (tfa MovingAverage, train.py:117-119)
//   lr  = CosineLrSchedule(step)                      (train.py:35-63)
//   optional: a non-finite gradient norm skips the update (SURVEY §5 failure detection; off by
//   default, the reference applies it)
// plus the fp32 -> compute-dtype weight cast, drop-connect masks and device step counter.
#include <algorithm>

#include "common.hpp"

namespace edet {

__device__ float sched_lr(const edet_sched& s, int step) {
  if (s.fixed_lr > 0.f) return s.fixed_lr;
  const float fs = (float)step;
  if (step < s.warmup_steps)
    return s.warmup_init + (fs / (float)s.warmup_steps) * (s.adjusted_lr - s.warmup_init);
  const float decay = (float)(s.total_steps - s.warmup_steps);
  return 0.5f * s.adjusted_lr * (1.f + cosf(3.14159265358979323846f * fs / decay));
}

// Norm pass.  Exactly EDET_OPT_NORM_BLOCKS blocks, each writing its two partial sums to its
// own slots (fp64, no atomics): the apply pass folds the slots in one fixed order, so every
// data-parallel replica holding the same all-reduced gradient computes the same gnorm bit for
// bit and the clip factor -- and hence the parameters -- never drift between replicas.
__global__ __launch_bounds__(256) void k_opt_norm(const float* w, const float* g, int64_t n, int64_t n_l2,
                                                  edet_sched sc, float* scalars, double* partials, int32_t* step) {
  __shared__ float red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gs = 0.f, ws = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float gv = g[i];
    if (i < n_l2) {
      const float wv = w[i];
      gv += sc.l2_weight * wv;
      ws += wv * wv;
    }
    gs += gv * gv;
  }
  gs = wave_sum(gs);
  ws = wave_sum(ws);
  if (lane == 0) { red[0][wave] = gs; red[1][wave] = ws; }
  __syncthreads();
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = (double)red[0][0] + red[0][1] + red[0][2] + red[0][3];
    partials[EDET_OPT_NORM_BLOCKS + blockIdx.x] = (double)red[1][0] + red[1][1] + red[1][2] + red[1][3];
    if (blockIdx.x == 0) {
      const int s = *step;
      scalars[4] = sched_lr(sc, s);
      *step = s + 1;
    }
  }
}

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sum of the norm partials, fixed order (thread t owns slot t; wave trees; waves 0..3)
__device__ double2 fold_partials(const double* partials) {
  static_assert(EDET_OPT_NORM_BLOCKS == 256, "one slot per thread");
  __shared__ double red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double a = wave_sum64(partials[threadIdx.x]);
  const double b = wave_sum64(partials[EDET_OPT_NORM_BLOCKS + threadIdx.x]);
  if (lane == 0) { red[0][wave] = a; red[1][wave] = b; }
  __syncthreads();
  return make_double2(((red[0][0] + red[0][1]) + red[0][2]) + red[0][3], ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3]);
}

template <typename T>
__global__ __launch_bounds__(256) void k_opt_apply(float* w, const float* g, float* v, float* ema, int64_t n,
                                                   int64_t n_l2, edet_sched sc, float* scalars,
                                                   const double* partials, T* wc, int32_t* step) {
  const double2 sums = fold_partials(partials);
  const float gnorm = (float)sqrt(sums.x);
  // every block folds the same partials, so every block takes the same branch
  if (sc.skip_nonfinite && !isfinite(sums.x)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      scalars[1] = (float)sums.x;
      scalars[2] = (float)sums.y;
      scalars[3] = gnorm;
      scalars[0] += (float)((double)sc.l2_weight * 0.5 * sums.y);
      scalars[6] = 1.f;
      if (step) *step -= 1;  // the learning-rate schedule does not advance over a skipped step
    }
    return;
  }
  const float clip = sc.clip_norm / fmaxf(gnorm, sc.clip_norm);
  const float lr = scalars[4];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float wv = w[i];
    float gv = g[i];
    if (i < n_l2) gv += sc.l2_weight * wv;
    gv *= clip;
    const float vv = sc.momentum * v[i] - lr * gv;
    v[i] = vv;
    wv += vv;
    w[i] = wv;
    if (ema) ema[i] -= (1.f - sc.ema_decay) * (ema[i] - wv);
    if (wc) wc[i] = from_f<T>(wv);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    scalars[1] = (float)sums.x;
    scalars[2] = (float)sums.y;
    scalars[3] = gnorm;
    scalars[0] += (float)((double)sc.l2_weight * 0.5 * sums.y);
    scalars[6] = 0.f;
  }
}

template <typename T>
__global__ void k_cast(const float* src, T* dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dst[i] = from_f<T>(src[i]);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// drop_connect.py:13-18: binary = floor(p + U[0,1)); output scale = binary / p
__global__ void k_dropmask(float* out, int n, float p, uint64_t seed, const int32_t* step) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = splitmix64(seed ^ splitmix64(((uint64_t)(uint32_t)*step << 32) | (uint32_t)i));
  const float u = (float)(h >> 40) * (1.f / 16777216.f);
  out[i] = floorf(p + u) / p;
}

// [N][K] fp32 master 1x1 kernels -> [K][ldN] compute-dtype copies (ldN = roundup(N, 8)), used
// as the B operand of the data-gradient GEMM.  table[e] = {src_off, dst_off, N, K}.
template <typename T>
__global__ __launch_bounds__(256) void k_transpose_cast(const float* src, T* dst, const int64_t* table) {
  __shared__ float tile[32][33];
  const int64_t* e = table + 4 * blockIdx.y;
  const int N = (int)e[2], K = (int)e[3];
  const int tk = cdiv(K, 32);
  const int tiles = cdiv(N, 32) * tk;
  if ((int)blockIdx.x >= tiles) return;
  const int n0 = (blockIdx.x / tk) * 32, k0 = (blockIdx.x % tk) * 32;
  const float* S = src + e[0];
  T* D = dst + e[1];
  const int ldn = cdiv(N, 8) * 8;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int n = n0 + r, k = k0 + tx;
    tile[r][tx] = (n < N && k < K) ? S[(size_t)n * K + k] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int k = k0 + r, n = n0 + tx;
    if (k < K && n < ldn) D[(size_t)k * ldn + n] = from_f<T>(n < N ? tile[tx][r] : 0.f);
  }
}

static int grid_for(int64_t n) {
  int64_t nb = (n + 255) / 256;
  if (nb > 2048) nb = 2048;
  if (nb < 1) nb = 1;
  return (int)nb;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_opt_norm(const float* w, const float* g, int64_t n, int64_t n_l2,
                  const edet_sched* sched, float* scalars, double* partials, int32_t* step,
                  edet_stream_t stream) {
  EDET_REQUIRE(w && g && sched && scalars && partials && step && n_l2 <= n, "opt_norm: bad argument");
  EDET_LAUNCH(k_opt_norm, dim3(EDET_OPT_NORM_BLOCKS), dim3(256), 0, (hipStream_t)stream, w, g, n, n_l2,
                     *sched, scalars, partials, step);
  return check_launch("edet opt_norm");
}

int edet_opt_apply(float* w, const float* g, float* v, float* ema, int64_t n, int64_t n_l2,
                   const edet_sched* sched, float* scalars, const double* partials, int dtype, void* wcompute,
                   int32_t* step, edet_stream_t stream) {
  EDET_REQUIRE(w && g && v && sched && scalars && partials && n_l2 <= n, "opt_apply: bad argument");
  EDET_DTYPE_DISPATCH(dtype, T, {
    EDET_LAUNCH(k_opt_apply<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, w, g, v, ema, n,
                       n_l2, *sched, scalars, partials, (T*)wcompute, step);
    return check_launch("edet opt_apply");
  });
}

int edet_cast_f32(int dtype, const float* src, void* dst, int64_t n, edet_stream_t stream) {
  EDET_REQUIRE(src && dst, "cast_f32: null argument");
  if (n <= 0) return EDET_OK;
  EDET_DTYPE_DISPATCH(dtype, T, {
    EDET_LAUNCH(k_cast<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, src, (T*)dst, n);
    return check_launch("edet cast");
  });
}

int edet_transpose_cast(int dtype, const float* src, void* dst, const int64_t* table, int n_entries,
                        int max_tiles, edet_stream_t stream) {
  EDET_REQUIRE(src && dst && table && n_entries >= 0 && max_tiles >= 0, "transpose_cast: bad argument");
  if (n_entries == 0 || max_tiles == 0) return EDET_OK;
  EDET_DTYPE_DISPATCH(dtype, T, {
    EDET_LAUNCH(k_transpose_cast<T>, dim3(max_tiles, n_entries), dim3(256), 0, (hipStream_t)stream, src,
                       (T*)dst, table);
    return check_launch("edet transpose_cast");
  });
}

int edet_dropmask(float* out, int n, float survival, uint64_t seed, const int32_t* step,
                  edet_stream_t stream) {
  EDET_REQUIRE(out && step && survival > 0.f, "dropmask: bad argument");
  if (n <= 0) return EDET_OK;
  EDET_LAUNCH(k_dropmask, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, n, survival, seed,
                     step);
  return check_launch("edet dropmask");
}

}  // extern "C"
