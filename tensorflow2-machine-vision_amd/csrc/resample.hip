// Stem convolution, max-pool resampling and BiFPN weighted fusion.
//
//   stem   : Conv2D 3x3 s2 SAME, no bias (layers/stem.py:15-22,38) + BN statistics
//   maxpool: MaxPooling2D 3x3 s2 SAME (layers/resample_feature_map.py:35-38); padded cells
//            are ignored; backward routes each window's gradient to its first maximum in
//            row-major window order (TF MaxPoolGrad semantics)
//   fuse   : BiFPNNode.call (layers/bifpn.py:59-65): out = sum_i R_i(v_i) * w_i / (sum w + 1e-4)
//            with R_i in {identity, nearest resize (tf.image.resize, half-pixel centres),
//            max-pool}; weights unconstrained (no ReLU)
#include <float.h>
#include <algorithm>
#include "common.hpp"

namespace edet {

// ------------------------------------------------------------------ stem
template <typename T>
__global__ __launch_bounds__(256) void k_stem_fwd(const T* x, int B, int H, int W, const T* w, int Cout,
                                                  T* y, double* sum, double* sq) {
  __shared__ float ws[27 * 64];
  __shared__ float red[2][4][64];  // [sum|sq][wave][channel]: fixed-order block reduction
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 27 * Cout; i += 256) ws[i] = to_f<T>(w[i]);
  __syncthreads();
  const int OH = cdiv(H, 2), OW = cdiv(W, 2);
  const int pt = same_pad(H, 3, 2), pl = same_pad(W, 3, 2);
  const long p = (long)blockIdx.x * 256 + tid;
  const bool valid = p < (long)B * OH * OW;
  float xin[27];
  if (valid) {
    const int n = (int)(p / ((long)OH * OW));
    const int rem = (int)(p - (long)n * OH * OW);
    const int oy = rem / OW, ox = rem - oy * OW;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iy = oy * 2 - pt + kh, ix = ox * 2 - pl + kw;
        const bool in = iy >= 0 && iy < H && ix >= 0 && ix < W;
        const T* px = x + (((size_t)n * H + iy) * W + ix) * 3;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) xin[(kh * 3 + kw) * 3 + ci] = in ? to_f<T>(px[ci]) : 0.f;
      }
  } else {
#pragma unroll
    for (int i = 0; i < 27; ++i) xin[i] = 0.f;
  }
  for (int co0 = 0; co0 < Cout; co0 += 8) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 27; ++k) {
      const float xv = xin[k];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += xv * ws[k * Cout + co0 + j];
    }
    if (valid) st8(y + (size_t)p * Cout + co0, acc);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = valid ? acc[j] : 0.f;
      const float s = wave_sum(a), q = wave_sum(a * a);
      if (lane == 0) { red[0][wave][co0 + j] = s; red[1][wave][co0 + j] = q; }
    }
  }
  __syncthreads();
  if (tid < Cout) {
    stat_put(sum, tid, (double)((red[0][0][tid] + red[0][1][tid]) + (red[0][2][tid] + red[0][3][tid])));
    stat_put(sq, tid, (double)((red[1][0][tid] + red[1][1][tid]) + (red[1][2][tid] + red[1][3][tid])));
  }
}

// dw[kh][kw][ci][co] += sum_pixels x_patch * dy
template <typename T>
__global__ __launch_bounds__(256) void k_stem_wgrad(const T* x, int B, int H, int W, const T* dy, int Cout,
                                                    float* dw, long px_per_wg, float* part) {
  __shared__ float patch[64][28];
  __shared__ float dys[64][65];
  const int tid = threadIdx.x;
  const int OH = cdiv(H, 2), OW = cdiv(W, 2);
  const int pt = same_pad(H, 3, 2), pl = same_pad(W, 3, 2);
  const long total = (long)B * OH * OW;
  const long p_begin = (long)blockIdx.x * px_per_wg;
  const long p_end = min(total, p_begin + px_per_wg);
  const int NOUT = 27 * Cout;
  float acc[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) acc[i] = 0.f;
  for (long p0 = p_begin; p0 < p_end; p0 += 64) {
    __syncthreads();
    for (int e = tid; e < 64 * 27; e += 256) {
      const int px = e / 27, k = e - px * 27;
      const long p = p0 + px;
      float v = 0.f;
      if (p < p_end) {
        const int n = (int)(p / ((long)OH * OW));
        const int rem = (int)(p - (long)n * OH * OW);
        const int oy = rem / OW, ox = rem - oy * OW;
        const int kh = k / 9, kw = (k / 3) % 3, ci = k % 3;
        const int iy = oy * 2 - pt + kh, ix = ox * 2 - pl + kw;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = to_f<T>(x[(((size_t)n * H + iy) * W + ix) * 3 + ci]);
      }
      patch[px][k] = v;
    }
    for (int e = tid; e < 64 * (Cout / 8); e += 256) {  // 16-byte vectors of dy
      const int px = e / (Cout / 8), co = (e - px * (Cout / 8)) * 8;
      const long p = p0 + px;
      float v[8];
      if (p < p_end) ld8(dy + (size_t)p * Cout + co, v);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) dys[px][co + j] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int j = tid + i * 256;
      if (j < NOUT) {
        const int pk = j / Cout, co = j - pk * Cout;
        float a = 0.f;
#pragma unroll 8
        for (int px = 0; px < 64; ++px) a += patch[px][pk] * dys[px][co];
        acc[i] += a;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int j = tid + i * 256;
    if (j < NOUT) {
      if (part) part[(size_t)blockIdx.x * NOUT + j] = acc[i];
      else atomicAdd(dw + j, acc[i]);
    }
  }
}

// ------------------------------------------------------------------ stem on MFMA (bf16)
// The 3x3x3 patch is K = 27 (zero-padded to 32): exactly one v_mfma_f32_16x16x32_bf16 step.
// One block owns R output rows of one image and stages the 2R+1 input rows they need in LDS
// (16-byte loads when a row is 16-byte aligned).  Operands are swapped (A = the weights as
// [Cout][k], B = the patches as [k][pixel]) so each lane ends up with 4 consecutive output
// channels of one pixel: 8-byte stores, and BN statistics accumulate per lane over all the
// block's pixels before one cross-lane reduction.
__device__ __forceinline__ void stem_stage_rows(const uint16_t* x, int H, int W, int n, int iy0, int IR, int RLP,
                                                uint16_t* xs) {
  const int RL = W * 3;
  if ((W & 7) == 0) {
    const int vpr = RL / 8;
    for (int v = threadIdx.x; v < IR * vpr; v += blockDim.x) {
      const int i = v / vpr, j = v - i * vpr, iy = iy0 + i;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (iy >= 0 && iy < H) val = *reinterpret_cast<const uint4*>(x + ((size_t)n * H + iy) * RL + j * 8);
      *reinterpret_cast<uint4*>(xs + i * RLP + j * 8) = val;
    }
  } else {
    for (int e = threadIdx.x; e < IR * RL; e += blockDim.x) {
      const int i = e / RL, j = e - i * RL, iy = iy0 + i;
      xs[i * RLP + j] = (iy >= 0 && iy < H) ? x[((size_t)n * H + iy) * RL + j] : (uint16_t)0;
    }
  }
}

// tap k = (kh*3 + kw)*3 + ci of output pixel (ry, ox) inside the staged rows (0 outside)
__device__ __forceinline__ uint16_t stem_tap(const uint16_t* xs, int RLP, int W, int pl, int ry, int ox, int k) {
  if (k >= 27) return 0;
  const int kh = k / 9, kw = (k / 3) % 3, ci = k % 3;
  const int ix = 2 * ox - pl + kw;
  if (ix < 0 || ix >= W) return 0;
  return xs[(2 * ry + kh) * RLP + ix * 3 + ci];
}

template <int NT>
__global__ __launch_bounds__(256) void k_stem2_fwd(const uint16_t* x, int B, int H, int W, const uint16_t* w, int Cout,
                                                   uint16_t* y, double* sum, double* sq, int R) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  __shared__ float red[2][4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g4 = lane >> 4;
  const int OH = cdiv(H, 2), OW = cdiv(W, 2);
  const int pt = same_pad(H, 3, 2), pl = same_pad(W, 3, 2);
  const int strips = cdiv(OH, R);
  const int n = blockIdx.x / strips, oy0 = (blockIdx.x - n * strips) * R;
  const int RLP = cdiv(W * 3, 8) * 8;
  stem_stage_rows(x, H, W, n, oy0 * 2 - pt, 2 * R + 1, RLP, xs);
  // A fragments: weights W[k][co] (HWIO), lane: k = 8*g4 .. +7, co = t*16 + lane%16
  bf16x8_t wa[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    uint16_t e8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * g4 + e;
      e8[e] = k < 27 ? w[k * Cout + t * 16 + (lane & 15)] : (uint16_t)0;
    }
    wa[t] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(e8));
  }
  __syncthreads();
  const int rows = min(R, OH - oy0);
  const int P = rows * OW;
  float s[NT][4], q[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) s[t][r] = q[t][r] = 0.f;
  const size_t pix0 = ((size_t)n * OH + oy0) * OW;
  for (int tile = wave; tile * 16 < P; tile += 4) {
    const int pix = tile * 16 + (lane & 15);
    const bool valid = pix < P;
    const int ry = valid ? pix / OW : 0, ox = valid ? pix - ry * OW : 0;
    uint16_t b8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) b8[e] = valid ? stem_tap(xs, RLP, W, pl, ry, ox, 8 * g4 + e) : (uint16_t)0;
    const bf16x8_t bf = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(b8));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      floatx4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[t], bf, floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      if (valid) {
        uint32_t lo = (uint32_t)f2bf(acc[0]) | ((uint32_t)f2bf(acc[1]) << 16);
        uint32_t hi = (uint32_t)f2bf(acc[2]) | ((uint32_t)f2bf(acc[3]) << 16);
        *reinterpret_cast<uint2*>(y + (pix0 + pix) * Cout + t * 16 + 4 * g4) = make_uint2(lo, hi);
#pragma unroll
        for (int r = 0; r < 4; ++r) { s[t][r] += acc[r]; q[t][r] += acc[r] * acc[r]; }
      }
    }
  }
  // reduce over the 16 pixel lanes that share a channel group, then over the 4 waves
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = s[t][r], b = q[t][r];
      a = row16_sum(a);
      b = row16_sum(b);
      if ((lane & 15) == 0) {
        red[0][wave][t * 16 + 4 * g4 + r] = a;
        red[1][wave][t * 16 + 4 * g4 + r] = b;
      }
    }
  __syncthreads();
  if (tid < Cout) {
    stat_put(sum, tid, (double)((red[0][0][tid] + red[0][1][tid]) + (red[0][2][tid] + red[0][3][tid])));
    stat_put(sq, tid, (double)((red[1][0][tid] + red[1][1][tid]) + (red[1][2][tid] + red[1][3][tid])));
  }
}

// dW[k][co] = sum_pixels patch[pixel][k] * dy[pixel][co]: D = A (patches^T, [k][pixel]) x
// B (dy, [pixel][co]) over 32-pixel steps.  Persistent over row strips; each block writes one
// [27][Cout] partial (summed in a fixed order afterwards).
template <int NT>
__global__ __launch_bounds__(256) void k_stem2_wgrad(const uint16_t* x, int B, int H, int W, const uint16_t* dy,
                                                     int Cout, float* part, int R) {
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g4 = lane >> 4;
  const int OH = cdiv(H, 2), OW = cdiv(W, 2);
  const int pt = same_pad(H, 3, 2), pl = same_pad(W, 3, 2);
  const int strips = cdiv(OH, R), total = B * strips;
  const int RLP = cdiv(W * 3, 8) * 8;
  const int DLD = Cout + 8;
  uint16_t* ds = xs + (2 * R + 1) * RLP;  // [R*OW][DLD]
  floatx4 acc[2][NT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int st = blockIdx.x; st < total; st += gridDim.x) {
    const int n = st / strips, oy0 = (st - n * strips) * R;
    const int rows = min(R, OH - oy0), P = rows * OW;
    __syncthreads();  // previous strip's readers are done
    stem_stage_rows(x, H, W, n, oy0 * 2 - pt, 2 * R + 1, RLP, xs);
    const uint16_t* dsrc = dy + ((size_t)n * OH + oy0) * OW * Cout;
    const int vpp = Cout / 8;
    for (int v = tid; v < R * OW * vpp; v += 256) {
      const int p = v / vpp, j = (v - p * vpp) * 8;
      uint4 val = make_uint4(0, 0, 0, 0);
      if (p < P) val = *reinterpret_cast<const uint4*>(dsrc + (size_t)p * Cout + j);
      *reinterpret_cast<uint4*>(ds + p * DLD + j) = val;
    }
    __syncthreads();
    for (int c32 = wave; c32 * 32 < P; c32 += 4) {
      bf16x8_t af[2], bf[NT];
#pragma unroll
      for (int i = 0; i < 2; ++i) {  // A: row k = i*16 + lane%16, pixels 8*g4 .. +7 of this step
        uint16_t e8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int pix = c32 * 32 + 8 * g4 + e;
          const int ry = pix / OW, ox = pix - ry * OW;
          e8[e] = pix < P ? stem_tap(xs, RLP, W, pl, ry, ox, i * 16 + (lane & 15)) : (uint16_t)0;
        }
        af[i] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(e8));
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {  // B: pixels 8*g4 .. +7, column co = t*16 + lane%16
        uint16_t e8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {  // rows past P are not staged (0 * garbage may be NaN)
          const int pix = c32 * 32 + 8 * g4 + e;
          e8[e] = pix < P ? ds[pix * DLD + t * 16 + (lane & 15)] : (uint16_t)0;
        }
        bf[t] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(e8));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[t], acc[i][t], 0, 0, 0);
    }
  }
  // reduce the four waves' accumulators (fixed order) and write this block's partial
  __syncthreads();
  float* red = reinterpret_cast<float*>(xs);  // [4][32][Cout]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        red[(wave * 32 + i * 16 + 4 * g4 + r) * Cout + t * 16 + (lane & 15)] = acc[i][t][r];
  __syncthreads();
  for (int e = tid; e < 27 * Cout; e += 256)
    part[(size_t)blockIdx.x * 27 * Cout + e] = (red[e] + red[32 * Cout + e]) + (red[64 * Cout + e] + red[96 * Cout + e]);
}

// ------------------------------------------------------------------ resample helpers
// tf.image.resize(method='nearest'): ResizeNearestNeighbor(align_corners=False,
// half_pixel_centers=True): in = min(floor((o + 0.5) * in/out), in - 1)
__device__ __forceinline__ int nearest_src(int o, int in, int out) {
  const float scale = (float)in / (float)out;
  int i = (int)floorf(((float)o + 0.5f) * scale);
  if (i > in - 1) i = in - 1;
  if (i < 0) i = 0;
  return i;
}

template <typename T>
__device__ __forceinline__ void lazy_load8(const edet_lazy& lz, const float2* af, size_t row, int c, int nc, float* o) {
  ld8m((const T*)lz.x + row * lz.ld + c, nc, o);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = lazy_apply(o[j], af[j], lz.act);
}

// max over the 3x3 s2 SAME window of output (oy, ox); optionally the argmax (row-major first)
template <typename T>
__device__ __forceinline__ void pool_window(const edet_lazy& lz, const float2* af, size_t img_row0, int H, int W,
                                            int pt, int pl, int oy, int ox, int c, int nc, float* best, int* arg,
                                            int* tap = nullptr) {
  int tk[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -FLT_MAX; arg[j] = -1; tk[j] = 0; }
  if (nc < 8) {  // channel tail (not reached with C % 8 == 0)
    for (int kh = 0; kh < 3; ++kh) {
      const int iy = oy * 2 - pt + kh;
      if (iy < 0 || iy >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int ix = ox * 2 - pl + kw;
        if (ix < 0 || ix >= W) continue;
        float v[8];
        lazy_load8<T>(lz, af, img_row0 + (size_t)iy * W + ix, c, nc, v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (arg[j] < 0 || v[j] > best[j]) { best[j] = v[j]; arg[j] = iy * W + ix; tk[j] = kh * 3 + kw; }
      }
    }
    if (tap)
#pragma unroll
      for (int j = 0; j < 8; ++j) tap[j] = tk[j];
    return;
  }
  // all nine taps are loaded first (select-predicated addresses: a load inside a divergent
  // `if` is waited on inside it), then scanned in the same row-major order
  float v[9][8];
  bool in[9];
  const T* X = (const T*)lz.x + img_row0 * lz.ld + c;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int iy = oy * 2 - pt + k / 3, ix = ox * 2 - pl + k % 3;
    in[k] = iy >= 0 && iy < H && ix >= 0 && ix < W;
    ld8(X + (in[k] ? (size_t)(iy * W + ix) * lz.ld : 0), v[k]);
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    if (!in[k]) continue;
    const int pos = (oy * 2 - pt + k / 3) * W + (ox * 2 - pl + k % 3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = lazy_apply(v[k][j], af[j], lz.act);
      if (arg[j] < 0 || t > best[j]) { best[j] = t; arg[j] = pos; tk[j] = k; }
    }
  }
  if (tap)
#pragma unroll
    for (int j = 0; j < 8; ++j) tap[j] = tk[j];
}

// the 8 window taps of a stored argmax vector (one byte per channel)
__device__ __forceinline__ void load_taps(const uint8_t* p, int* tap) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    tap[j] = (w.x >> (8 * j)) & 0xff;
    tap[4 + j] = (w.y >> (8 * j)) & 0xff;
  }
}
__device__ __forceinline__ void store_taps(uint8_t* p, const int* tap) {
  uint2 w = make_uint2(0u, 0u);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    w.x |= (uint32_t)tap[j] << (8 * j);
    w.y |= (uint32_t)tap[4 + j] << (8 * j);
  }
  *reinterpret_cast<uint2*>(p) = w;
}

// per-channel lazy-BN affine of each input, once per block into LDS (was recomputed per
// element: four global loads plus the fp64 mean/var per channel per pixel)
__device__ __forceinline__ void load_affine(const edet_lazy& lz, int C, float inv, float2* tab) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) tab[c] = bn_affine(lz.bn, 0, c, inv);
}
__device__ __forceinline__ void affine8_lds(const float2* tab, int c, float2* af) {
#pragma unroll
  for (int j = 0; j < 8; ++j) af[j] = tab[c + j];
}

__device__ __forceinline__ void affine8(const edet_lazy& lz, int c, int C, float inv, float2* af) {
#pragma unroll
  for (int j = 0; j < 8; ++j) af[j] = (c + j < C) ? bn_affine(lz.bn, 0, c + j, inv) : make_float2(1.f, 0.f);
}

template <typename T>
__global__ __launch_bounds__(256) void k_maxpool_fwd(edet_lazy lz, int B, int H, int W, int C, T* y,
                                                     uint8_t* taps) {
  extern __shared__ float2 aft[];  // [C]
  load_affine(lz, C, 1.f / (float)(B * H * W), aft);
  __syncthreads();
  const int OH = cdiv(H, 2), OW = cdiv(W, 2), nv = C / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * OH * OW * nv) return;
  const int cv = (int)(idx % nv);
  const long pix = idx / nv;
  const int n = (int)(pix / ((long)OH * OW));
  const int rem = (int)(pix - (long)n * OH * OW);
  const int oy = rem / OW, ox = rem - oy * OW;
  float2 af[8];
  affine8_lds(aft, cv * 8, af);
  float best[8];
  int arg[8], tap[8];
  pool_window<T>(lz, af, (size_t)n * H * W, H, W, same_pad(H, 3, 2), same_pad(W, 3, 2), oy, ox, cv * 8, 8, best, arg,
                 tap);
  st8(y + (size_t)pix * C + cv * 8, best);
  if (taps) store_taps(taps + (size_t)pix * C + cv * 8, tap);
}

// max-pool backward from the forward's recorded window taps (edet_maxpool_bwd_taps, round 6):
// an input pixel's <= 2 x 2 covering windows are read at once -- taps and dy, no input values,
// no BN tables -- instead of re-evaluating up to four 3 x 3 windows one after another
// (resample_p6/p7: 16 -> a few us per call)
template <typename T>
__global__ __launch_bounds__(256) void k_maxpool_bwd_taps(int B, int H, int W, int C, const uint8_t* taps,
                                                          const T* dy, T* dx, int accumulate) {
  const int OH = cdiv(H, 2), OW = cdiv(W, 2), nv = C / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H * W * nv) return;
  const int cv = (int)(idx % nv), c = cv * 8;
  const long pix = idx / nv;
  const int n = (int)(pix / ((long)H * W));
  const int rem = (int)(pix - (long)n * H * W);
  const int iy = rem / W, ix = rem - iy * W;
  const int pt = same_pad(H, 3, 2), pl = same_pad(W, 3, 2);
  const int oy_lo = max(0, fdiv(iy + pt - 1, 2)), oy_hi = min(OH - 1, fdiv(iy + pt, 2));
  const int ox_lo = max(0, fdiv(ix + pl - 1, 2)), ox_hi = min(OW - 1, fdiv(ix + pl, 2));
  const size_t o0 = (size_t)n * OH * OW;
  uint2 tq[4];
  float g[4][8];
  bool ok[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // every window's loads issued before any is used
    const int oy = oy_lo + (k >> 1), ox = ox_lo + (k & 1);
    ok[k] = oy <= oy_hi && ox <= ox_hi;
    const size_t o = (o0 + (ok[k] ? (size_t)oy * OW + ox : 0)) * C + c;
    tq[k] = *reinterpret_cast<const uint2*>(taps + o);
    ld8(dy + o, g[k]);
  }
  float d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // windows in row-major order (the recompute path's order)
    if (!ok[k]) continue;
    const int oy = oy_lo + (k >> 1), ox = ox_lo + (k & 1);
    const int kme = (iy - (oy * 2 - pt)) * 3 + (ix - (ox * 2 - pl));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int tap = (int)(((j < 4 ? tq[k].x : tq[k].y) >> (8 * (j & 3))) & 0xffu);
      if (tap == kme) d[j] += g[k][j];
    }
  }
  acc8m(dx + (size_t)pix * C + c, 8, d, accumulate);
}

// gather form of the max-pool backward: input pixel collects dy of every window whose
// (recomputed) argmax is this pixel
// (or, given the forward's stored taps `parg`, reads them instead of re-evaluating windows)
template <typename T>
__device__ __forceinline__ void pool_bwd_gather(const edet_lazy& lz, const float2* af, const T* dy, size_t img_row0,
                                                size_t out_row0, int H, int W, int OH, int OW, int C, int iy, int ix,
                                                int c, float scale, float* d, const uint8_t* parg = nullptr) {
  const int pt = same_pad(H, 3, 2), pl = same_pad(W, 3, 2);
  const int oy_lo = max(0, fdiv(iy + pt - 2 + 1, 2)), oy_hi = min(OH - 1, fdiv(iy + pt, 2));
  const int ox_lo = max(0, fdiv(ix + pl - 2 + 1, 2)), ox_hi = min(OW - 1, fdiv(ix + pl, 2));
  const int me = iy * W + ix;
  if (parg) {
    for (int oy = oy_lo; oy <= oy_hi; ++oy)
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const size_t o = out_row0 + (size_t)oy * OW + ox;
        int tap[8];
        load_taps(parg + o * C + c, tap);
        float g[8];
        ld8(dy + o * C + c, g);
        const int kme = (iy - (oy * 2 - pt)) * 3 + (ix - (ox * 2 - pl));
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (tap[j] == kme) d[j] += g[j] * scale;
      }
    return;
  }
  for (int oy = oy_lo; oy <= oy_hi; ++oy)
    for (int ox = ox_lo; ox <= ox_hi; ++ox) {
      float best[8];
      int arg[8];
      pool_window<T>(lz, af, img_row0, H, W, pt, pl, oy, ox, c, 8, best, arg);
      float g[8];
      ld8(dy + (out_row0 + (size_t)oy * OW + ox) * C + c, g);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (arg[j] == me) d[j] += g[j] * scale;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void k_maxpool_bwd(edet_lazy lz, int B, int H, int W, int C, const T* dy, T* dx,
                                                     int accumulate) {
  extern __shared__ float2 aft[];  // [C]
  load_affine(lz, C, 1.f / (float)(B * H * W), aft);
  __syncthreads();
  const int OH = cdiv(H, 2), OW = cdiv(W, 2), nv = C / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)B * H * W * nv) return;
  const int cv = (int)(idx % nv);
  const long pix = idx / nv;
  const int n = (int)(pix / ((long)H * W));
  const int rem = (int)(pix - (long)n * H * W);
  const int iy = rem / W, ix = rem - iy * W;
  float2 af[8];
  affine8_lds(aft, cv * 8, af);
  float d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = 0.f;
  pool_bwd_gather<T>(lz, af, dy, (size_t)n * H * W, (size_t)n * OH * OW, H, W, OH, OW, C, iy, ix, cv * 8, 1.f, d);
  acc8m(dx + (size_t)pix * C + cv * 8, 8, d, accumulate);
}

// ------------------------------------------------------------------ BiFPN fusion
struct FuseArgs {
  edet_fuse_input in[3];
  const float* w;
  const void* fused;
  const void* dout;
  void* out;
  float* dw;
  int n_in, B, H, W, C;
  int nb_w, nb_in[3];
};

// resampled value of input i at output pixel (n, h, w), 8 channels from c
// MAXPOOL with fi.pool_arg: `store` (forward) writes the window taps of output pixel `pix`;
// otherwise (backward) they are read and only the 8 winning taps are loaded and transformed
template <typename T>
__device__ __forceinline__ void fuse_input_value(const edet_fuse_input& fi, const float2* af, int n, int h, int w,
                                                 int OH, int OW, int c, float* v, size_t pix = 0, int C = 0,
                                                 bool store = false) {
  const int Hi = fi.H, Wi = fi.W;
  const size_t r0 = (size_t)n * Hi * Wi;
  if (fi.mode == EDET_MODE_SAME) {
    lazy_load8<T>(fi.v, af, r0 + (size_t)h * Wi + w, c, 8, v);
  } else if (fi.mode == EDET_MODE_UPSAMPLE) {
    const int iy = nearest_src(h, Hi, OH), ix = nearest_src(w, Wi, OW);
    lazy_load8<T>(fi.v, af, r0 + (size_t)iy * Wi + ix, c, 8, v);
  } else if (fi.pool_arg && !store) {
    int tap[8];
    load_taps(fi.pool_arg + pix * C + c, tap);
    const int y0 = h * 2 - same_pad(Hi, 3, 2), x0 = w * 2 - same_pad(Wi, 3, 2);
    const T* X = (const T*)fi.v.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const size_t row = r0 + (size_t)(y0 + tap[j] / 3) * Wi + (x0 + tap[j] % 3);
      v[j] = lazy_apply(to_f<T>(X[row * fi.v.ld + c + j]), af[j], fi.v.act);
    }
  } else {
    int arg[8], tap[8];
    pool_window<T>(fi.v, af, r0, Hi, Wi, same_pad(Hi, 3, 2), same_pad(Wi, 3, 2), h, w, c, 8, v, arg, tap);
    if (store && fi.pool_arg) store_taps(fi.pool_arg + pix * C + c, tap);
  }
}

__device__ __forceinline__ float fuse_denom(const float* w, int n_in) {
  float s = 0.f;
  for (int i = 0; i < n_in; ++i) s += w[i];
  return s + 1e-4f;
}

template <typename T>
__global__ __launch_bounds__(256) void k_fuse_fwd(FuseArgs g) {
  extern __shared__ float2 aft[];  // [n_in][C]
  for (int i = 0; i < g.n_in; ++i)
    load_affine(g.in[i].v, g.C, 1.f / (float)(g.B * g.in[i].H * g.in[i].W), aft + i * g.C);
  __syncthreads();
  const int nv = g.C / 8;
  const long total = (long)g.B * g.H * g.W * nv;
  const float den = fuse_denom(g.w, g.n_in);
  // grid-stride over the vectors: a capped grid amortises the per-block affine tables
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int cv = (int)(idx % nv);
    const long pix = idx / nv;
    const int n = (int)(pix / ((long)g.H * g.W));
    const int rem = (int)(pix - (long)n * g.H * g.W);
    const int h = rem / g.W, w = rem - h * g.W;
    float o[8];
    for (int i = 0; i < g.n_in; ++i) {
      const edet_fuse_input& fi = g.in[i];
      float2 af[8];
      affine8_lds(aft + i * g.C, cv * 8, af);
      float v[8];
      fuse_input_value<T>(fi, af, n, h, w, g.H, g.W, cv * 8, v, (size_t)pix, g.C, true);
      const float wn = g.w[i] / den;  // one division per input, not per element
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = v[j] * wn;
        o[j] = (i == 0) ? t : o[j] + t;
      }
    }
    st8((T*)g.out + (size_t)pix * g.C + cv * 8, o);
  }
}

// bf16 forward with the input modes compile-time (M0..M2: EDET_MODE_*, M2 = -1: two inputs): every
// input's raw vectors of an output pixel are loaded before any is transformed, so a thread has
// all its inputs' round trips in flight at once (the runtime mode loop loaded, waited for and
// transformed one input at a time: three serial round trips per vector at a bottom-up node).
// Same values, same order of the weighted sum, same pool taps as k_fuse_fwd.
template <int M>
struct FuseRaw {
  uint4 r[M == EDET_MODE_MAXPOOL ? 9 : 1];
  uint32_t ok;
};
template <int M>
__device__ __forceinline__ void fuse_raw_load(FuseRaw<M>& s, const edet_fuse_input& fi, int n, int h, int w, int OH,
                                              int OW, int c) {
  const int Hi = fi.H, Wi = fi.W;
  const uint16_t* X = (const uint16_t*)fi.v.x + (size_t)n * Hi * Wi * fi.v.ld + c;
  if constexpr (M == EDET_MODE_SAME) {
    s.r[0] = gld16(X + (size_t)(h * Wi + w) * fi.v.ld);
  } else if constexpr (M == EDET_MODE_UPSAMPLE) {
    const int iy = nearest_src(h, Hi, OH), ix = nearest_src(w, Wi, OW);
    s.r[0] = gld16(X + (size_t)(iy * Wi + ix) * fi.v.ld);
  } else if constexpr (M == EDET_MODE_MAXPOOL) {
    const int y0 = h * 2 - same_pad(Hi, 3, 2), x0 = w * 2 - same_pad(Wi, 3, 2);
    s.ok = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int iy = y0 + k / 3, ix = x0 + k % 3;
      const bool in = iy >= 0 && iy < Hi && ix >= 0 && ix < Wi;
      s.r[k] = gld16(X + (in ? (size_t)(iy * Wi + ix) * fi.v.ld : 0));
      s.ok |= (uint32_t)in << k;
    }
  }
}
__device__ __forceinline__ void unpack_bf8(const uint4& q, float* o) {
  const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w4[i] << 16);
    o[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
  }
}
// ACT: the inputs' activation as a compile-time case (0 none, 1 swish) when every input of the
// node shares it, -1 = read fi.v.act (the runtime test per element sat in the pool's 72-value
// compare loop)
template <int ACT>
__device__ __forceinline__ float fuse_act(float x, float2 a, int act) {
  if constexpr (ACT < 0) {
    return lazy_apply(x, a, act);
  } else {
    const float u = x * a.x + a.y;
    return ACT == 1 ? swishf_(u) : u;
  }
}
template <int M, int ACT = -1>
__device__ __forceinline__ void fuse_raw_value(const FuseRaw<M>& s, const edet_fuse_input& fi, const float2* af,
                                               size_t pix, int C, int c, float* v) {
  if constexpr (M == EDET_MODE_MAXPOOL) {
    float best[8];
    int arg[8], tk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -FLT_MAX; arg[j] = -1; tk[j] = 0; }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!((s.ok >> k) & 1)) continue;
      float x[8];
      unpack_bf8(s.r[k], x);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float t = fuse_act<ACT>(x[j], af[j], fi.v.act);
        if (arg[j] < 0 || t > best[j]) { best[j] = t; arg[j] = k; tk[j] = k; }
      }
    }
    if (fi.pool_arg) store_taps(fi.pool_arg + pix * C + c, tk);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = best[j];
  } else {
    float x[8];
    unpack_bf8(s.r[0], x);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fuse_act<ACT>(x[j], af[j], fi.v.act);
  }
}
template <int M0, int M1, int M2, int ACT = -1>
__global__ __launch_bounds__(256) void k_fuse_fwd_m(FuseArgs g) {
  using T = uint16_t;
  extern __shared__ float2 aft[];  // [n_in][C]
  constexpr int NIN = 2 + (M2 >= 0);
  for (int i = 0; i < NIN; ++i)
    load_affine(g.in[i].v, g.C, 1.f / (float)(g.B * g.in[i].H * g.in[i].W), aft + i * g.C);
  __syncthreads();
  const int nv = g.C / 8;
  const long total = (long)g.B * g.H * g.W * nv;
  const float den = fuse_denom(g.w, NIN);
  float wn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) wn[i] = i < NIN ? g.w[i] / den : 0.f;  // one division per input
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int cv = (int)(idx % nv);
    const long pix = idx / nv;
    const int n = (int)(pix / ((long)g.H * g.W));
    const int rem = (int)(pix - (long)n * g.H * g.W);
    const int h = rem / g.W, w = rem - h * g.W;
    FuseRaw<M0> r0;
    FuseRaw<M1> r1;
    FuseRaw<M2 >= 0 ? M2 : EDET_MODE_SAME> r2;
    fuse_raw_load<M0>(r0, g.in[0], n, h, w, g.H, g.W, cv * 8);
    fuse_raw_load<M1>(r1, g.in[1], n, h, w, g.H, g.W, cv * 8);
    if constexpr (M2 >= 0) fuse_raw_load<M2>(r2, g.in[2], n, h, w, g.H, g.W, cv * 8);
    float o[8], v[8];
    float2 af[8];
    affine8_lds(aft, cv * 8, af);
    fuse_raw_value<M0, ACT>(r0, g.in[0], af, (size_t)pix, g.C, cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j] * wn[0];
    affine8_lds(aft + g.C, cv * 8, af);
    fuse_raw_value<M1, ACT>(r1, g.in[1], af, (size_t)pix, g.C, cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = o[j] + v[j] * wn[1];
    if constexpr (M2 >= 0) {
      affine8_lds(aft + 2 * g.C, cv * 8, af);
      fuse_raw_value<M2, ACT>(r2, g.in[2], af, (size_t)pix, g.C, cv * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = o[j] + v[j] * wn[2];
    }
    st8((T*)g.out + (size_t)pix * g.C + cv * 8, o);
  }
}

// the dx blocks of the fusion backward (input i's pixels: b counts from the first dx block)
template <typename T>
__device__ __forceinline__ void fuse_bwd_dx(const FuseArgs& g, const float2* aft, int b) {
  const int tid = threadIdx.x;
  const int nv = g.C / 8;
  const float den = fuse_denom(g.w, g.n_in);
  int i = 0;
  for (; i < g.n_in - 1; ++i) {
    if (b < g.nb_in[i]) break;
    b -= g.nb_in[i];
  }
  const edet_fuse_input& fi = g.in[i];
  const int Hi = fi.H, Wi = fi.W;
  const long idx = (long)b * 256 + tid;
  if (idx >= (long)g.B * Hi * Wi * nv) return;
  const int cv = (int)(idx % nv);
  const long pix = idx / nv;
  const int n = (int)(pix / ((long)Hi * Wi));
  const int rem = (int)(pix - (long)n * Hi * Wi);
  const int iy = rem / Wi, ix = rem - iy * Wi;
  const float wn = g.w[i] / den;
  const T* dF = (const T*)g.dout;
  const size_t o0 = (size_t)n * g.H * g.W;
  float d[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = 0.f;
  if (fi.mode == EDET_MODE_SAME) {
    float v[8];
    ld8(dF + (o0 + (size_t)iy * g.W + ix) * g.C + cv * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = v[j] * wn;
  } else if (fi.mode == EDET_MODE_UPSAMPLE && g.H == 2 * Hi && g.W == 2 * Wi) {
    // exact x2 (the BiFPN's): input (iy, ix) is the nearest source of output rows 2iy, 2iy+1 and
    // columns 2ix, 2ix+1 -- four loads at once (the window walk below waited for each in turn)
    uint4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      q[k] = gld16(dF + (o0 + (size_t)(2 * iy + (k >> 1)) * g.W + 2 * ix + (k & 1)) * g.C + cv * 8);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float v[8];
      if constexpr (sizeof(T) == 2) {
        const uint32_t w4[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] = __uint_as_float(w4[e] << 16);
          v[2 * e + 1] = __uint_as_float(w4[e] & 0xffff0000u);
        }
      } else {
        ld8(dF + (o0 + (size_t)(2 * iy + (k >> 1)) * g.W + 2 * ix + (k & 1)) * g.C + cv * 8, v);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += v[j] * wn;
    }
  } else if (fi.mode == EDET_MODE_UPSAMPLE) {
    // output rows h with nearest_src(h) == iy lie in [iy*OH/Hi - 1, (iy+1)*OH/Hi + 1]
    const int h_lo = max(0, (int)((long)iy * g.H / Hi) - 1), h_hi = min(g.H - 1, (int)((long)(iy + 1) * g.H / Hi) + 1);
    const int w_lo = max(0, (int)((long)ix * g.W / Wi) - 1), w_hi = min(g.W - 1, (int)((long)(ix + 1) * g.W / Wi) + 1);
    for (int h = h_lo; h <= h_hi; ++h) {
      if (nearest_src(h, Hi, g.H) != iy) continue;
      for (int w = w_lo; w <= w_hi; ++w) {
        if (nearest_src(w, Wi, g.W) != ix) continue;
        float v[8];
        ld8(dF + (o0 + (size_t)h * g.W + w) * g.C + cv * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] += v[j] * wn;
      }
    }
  } else if (fi.pool_arg) {
    // max-pooled input with the forward's taps: the (at most 2 x 2) outputs whose window holds
    // this pixel, their taps and dF loaded at once (pool_bwd_gather's loops waited for each)
    const int pt = same_pad(Hi, 3, 2), pl = same_pad(Wi, 3, 2);
    const int oy_lo = max(0, fdiv(iy + pt - 1, 2)), oy_hi = min(g.H - 1, fdiv(iy + pt, 2));
    const int ox_lo = max(0, fdiv(ix + pl - 1, 2)), ox_hi = min(g.W - 1, fdiv(ix + pl, 2));
    uint2 tq[4];
    uint4 dq[4];
    bool okk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int oy = oy_lo + (k >> 1), ox = ox_lo + (k & 1);
      okk[k] = oy <= oy_hi && ox <= ox_hi;
      const size_t o = o0 + (okk[k] ? (size_t)oy * g.W + ox : 0);
      tq[k] = *reinterpret_cast<const uint2*>(fi.pool_arg + o * g.C + cv * 8);
      dq[k] = gld16(dF + o * g.C + cv * 8);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!okk[k]) continue;
      const int oy = oy_lo + (k >> 1), ox = ox_lo + (k & 1);
      const int kme = (iy - (oy * 2 - pt)) * 3 + (ix - (ox * 2 - pl));
      float gv[8];
      if constexpr (sizeof(T) == 2) {
        const uint32_t w4[4] = {dq[k].x, dq[k].y, dq[k].z, dq[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gv[2 * e] = __uint_as_float(w4[e] << 16);
          gv[2 * e + 1] = __uint_as_float(w4[e] & 0xffff0000u);
        }
      } else {
        ld8(dF + (o0 + (size_t)oy * g.W + ox) * g.C + cv * 8, gv);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tap = (int)(((j < 4 ? tq[k].x : tq[k].y) >> (8 * (j & 3))) & 0xffu);
        if (tap == kme) d[j] += gv[j] * wn;
      }
    }
  } else {
    float2 af[8];
    affine8_lds(aft + i * g.C, cv * 8, af);
    pool_bwd_gather<T>(fi.v, af, dF, (size_t)n * Hi * Wi, o0, Hi, Wi, g.H, g.W, g.C, iy, ix, cv * 8, wn, d,
                       fi.pool_arg);
  }
  acc8m((T*)fi.dx + (size_t)pix * g.C + cv * 8, 8, d, fi.accumulate);
}

template <typename T>
__global__ __launch_bounds__(256) void k_fuse_bwd(FuseArgs g) {
  __shared__ float red[3][4];
  extern __shared__ float2 aft[];  // [n_in][C]
  for (int i = 0; i < g.n_in; ++i)
    load_affine(g.in[i].v, g.C, 1.f / (float)(g.B * g.in[i].H * g.in[i].W), aft + i * g.C);
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nv = g.C / 8;
  const float den = fuse_denom(g.w, g.n_in);
  int b = blockIdx.x;
  if (b < g.nb_w) {
    // weight gradient: dw_i = sum dF * (v_i - F) / den.  A bounded grid (<= 256 blocks)
    // walks the pixels and keeps partials in registers: one block per 256 vectors put
    // thousands of same-address atomics on the 3 weights.
    float part[3] = {0.f, 0.f, 0.f};
    const float rden = 1.f / den;
    const long total = (long)g.B * g.H * g.W * nv;
    for (long idx = (long)b * 256 + tid; idx < total; idx += (long)g.nb_w * 256) {
      const int cv = (int)(idx % nv);
      const long pix = idx / nv;
      const int n = (int)(pix / ((long)g.H * g.W));
      const int rem = (int)(pix - (long)n * g.H * g.W);
      const int h = rem / g.W, w = rem - h * g.W;
      float F[8], dF[8];
      ld8((const T*)g.fused + (size_t)pix * g.C + cv * 8, F);
      ld8((const T*)g.dout + (size_t)pix * g.C + cv * 8, dF);
      for (int i = 0; i < g.n_in; ++i) {
        const edet_fuse_input& fi = g.in[i];
        float2 af[8];
        affine8_lds(aft + i * g.C, cv * 8, af);
        float v[8];
        fuse_input_value<T>(fi, af, n, h, w, g.H, g.W, cv * 8, v, (size_t)pix, g.C, false);
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += dF[j] * (v[j] - F[j]);
        part[i] += s * rden;
      }
    }
    for (int i = 0; i < g.n_in; ++i) {
      const float s = wave_sum(part[i]);
      if (lane == 0) red[i][wave] = s;
    }
    __syncthreads();
    if (tid < g.n_in) atomicAdd(g.dw + tid, red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3]);
    return;
  }
  fuse_bwd_dx<T>(g, aft, b - g.nb_w);
}

// bf16 backward with compile-time input modes: the weight-gradient blocks load F, dF and every
// input's raw vectors of a pixel before any use (the runtime loop waited for each input in turn:
// with a bounded grid of long-lived blocks those serial round trips were the launch's tail, D4
// 130-138 us per call); a max-pooled input recomputes its 3x3 window (nine loads at once)
// instead of chaining a tap load and the tap-indexed rows.  The dx blocks are k_fuse_bwd's.
template <int M0, int M1, int M2, int ACT = -1>
__global__ __launch_bounds__(256) void k_fuse_bwd_m(FuseArgs g) {
  using T = uint16_t;
  __shared__ float red[3][4];
  extern __shared__ float2 aft[];  // [n_in][C]
  constexpr int NIN = 2 + (M2 >= 0);
  for (int i = 0; i < NIN; ++i)
    load_affine(g.in[i].v, g.C, 1.f / (float)(g.B * g.in[i].H * g.in[i].W), aft + i * g.C);
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nv = g.C / 8;
  const float den = fuse_denom(g.w, NIN);
  const int b = blockIdx.x;
  if (b >= g.nb_w) {
    fuse_bwd_dx<T>(g, aft, b - g.nb_w);
    return;
  }
  float part[3] = {0.f, 0.f, 0.f};
  const float rden = 1.f / den;
  const long total = (long)g.B * g.H * g.W * nv;
  for (long idx = (long)b * 256 + tid; idx < total; idx += (long)g.nb_w * 256) {
    const int cv = (int)(idx % nv);
    const long pix = idx / nv;
    const int n = (int)(pix / ((long)g.H * g.W));
    const int rem = (int)(pix - (long)n * g.H * g.W);
    const int h = rem / g.W, w = rem - h * g.W;
    const uint4 fr = gld16((const T*)g.fused + (size_t)pix * g.C + cv * 8);
    const uint4 dr = gld16((const T*)g.dout + (size_t)pix * g.C + cv * 8);
    FuseRaw<M0> r0;
    FuseRaw<M1> r1;
    FuseRaw<M2 >= 0 ? M2 : EDET_MODE_SAME> r2;
    fuse_raw_load<M0>(r0, g.in[0], n, h, w, g.H, g.W, cv * 8);
    fuse_raw_load<M1>(r1, g.in[1], n, h, w, g.H, g.W, cv * 8);
    if constexpr (M2 >= 0) fuse_raw_load<M2>(r2, g.in[2], n, h, w, g.H, g.W, cv * 8);
    float F[8], dF[8], v[8];
    unpack_bf8(fr, F);
    unpack_bf8(dr, dF);
    float2 af[8];
    auto acc = [&](int i) {
      float t = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) t += dF[j] * (v[j] - F[j]);
      part[i] += t * rden;
    };
    // (the pool taps are not stored from here: pool_arg belongs to the forward)
    edet_fuse_input f0 = g.in[0], f1 = g.in[1], f2 = g.in[NIN - 1];
    f0.pool_arg = nullptr; f1.pool_arg = nullptr; f2.pool_arg = nullptr;
    affine8_lds(aft, cv * 8, af);
    fuse_raw_value<M0, ACT>(r0, f0, af, (size_t)pix, g.C, cv * 8, v);
    acc(0);
    affine8_lds(aft + g.C, cv * 8, af);
    fuse_raw_value<M1, ACT>(r1, f1, af, (size_t)pix, g.C, cv * 8, v);
    acc(1);
    if constexpr (M2 >= 0) {
      affine8_lds(aft + 2 * g.C, cv * 8, af);
      fuse_raw_value<M2, ACT>(r2, f2, af, (size_t)pix, g.C, cv * 8, v);
      acc(2);
    }
  }
  for (int i = 0; i < NIN; ++i) {
    const float s = wave_sum(part[i]);
    if (lane == 0) red[i][wave] = s;
  }
  __syncthreads();
  if (tid < NIN) atomicAdd(g.dw + tid, red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3]);
}

// ------------------------------------------------------------------ fusion backward from d(value) (ABI 10)
// One pass over the node (bifpn.py:59-66 + OpAfterCombine's swish, :26) from the gradient of
// its VALUE dv = d act(F): dF = dv * act'(F) is formed in registers, so the separate
// d(value) -> d(raw) pass over the output and its re-reads by the dx and weight-gradient blocks
// are gone.  Two kinds of blocks:
//  * quad blocks: a thread owns a 2x2 output quad x 8 channels.  It loads dv and F of the quad,
//    every same-size input's raw vectors and the exact-x2 upsampled input's one source vector
//    (the quad's nearest source), writes the same-size inputs' dx (4 vectors each) and the
//    upsampled input's dx (the quad's sum, 1 vector), and adds dF * (v_i - F) per element.
//  * pool blocks (first, the heavier ones): a thread owns one pixel x 8 channels of the
//    max-pooled input; with the forward's recorded taps it gathers dF from the <= 2x2 windows
//    holding the pixel (dv and F loaded with the taps) and, for every window whose tap picks the
//    pixel, adds dF * (x(pixel) - F(window)): each output counted once, at its argmax.
// The weight gradient leaves as one float4 of per-input sums per block (fixed order, no
// atomics); edet_bifpn_fuse_fold sums them per node and divides by (sum w + 1e-4).
struct FuseDvArgs {
  edet_fuse_input in[3];
  const float* w;
  const void* fused;  // raw F [B*H*W][C]
  const void* dv;     // d(value) [B*H*W][C]
  float4* part;       // [blocks]
  int B, H, W, C, QH, QW;
  int nb_pool;  // pool blocks (the first ones); 0 without a max-pooled input
};

template <int OACT>
__device__ __forceinline__ void fuse_df(const uint4& dq, const uint4& fq, float* F, float* d) {
  unpack_bf8(fq, F);
  unpack_bf8(dq, d);
  if constexpr (OACT == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= dswishf_(F[j]);
  }
}

template <int M0, int M1, int M2, int ACT, int OACT>
__global__ __launch_bounds__(256) void k_fuse_bwd_dv(FuseDvArgs g) {
  using T = uint16_t;
  constexpr int NIN = 2 + (M2 >= 0);
  constexpr int MODE[3] = {M0, M1, M2};
  constexpr int PI = M2 == EDET_MODE_MAXPOOL ? 2 : (M1 == EDET_MODE_MAXPOOL ? 1 : -1);
  extern __shared__ float2 aft[];  // [n_in][C]
  __shared__ float red[3][4];
  for (int i = 0; i < NIN; ++i)
    load_affine(g.in[i].v, g.C, 1.f / (float)(g.B * g.in[i].H * g.in[i].W), aft + i * g.C);
  __syncthreads();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int C = g.C, nv = C / 8;
  const float den = fuse_denom(g.w, NIN);
  float wn[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) wn[i] = i < NIN ? g.w[i] / den : 0.f;
  float part[3] = {0.f, 0.f, 0.f};
  const T* Fp = (const T*)g.fused;
  const T* Dp = (const T*)g.dv;
  const int b = blockIdx.x;
  if constexpr (PI >= 0) {
    if (b < g.nb_pool) {
      const edet_fuse_input& fi = g.in[PI];
      const int Hi = fi.H, Wi = fi.W;
      const long idx = (long)b * 256 + tid;
      if (idx < (long)g.B * Hi * Wi * nv) {
        const int cv = (int)(idx % nv), c = cv * 8;
        const long pix = idx / nv;
        const int n = (int)(pix / ((long)Hi * Wi));
        const int rem = (int)(pix - (long)n * Hi * Wi);
        const int iy = rem / Wi, ix = rem - iy * Wi;
        const int pt = same_pad(Hi, 3, 2), pl = same_pad(Wi, 3, 2);
        const int oy_lo = max(0, fdiv(iy + pt - 1, 2)), oy_hi = min(g.H - 1, fdiv(iy + pt, 2));
        const int ox_lo = max(0, fdiv(ix + pl - 1, 2)), ox_hi = min(g.W - 1, fdiv(ix + pl, 2));
        const size_t o0 = (size_t)n * g.H * g.W;
        uint2 tq[4];
        uint4 dq[4], fq[4];
        bool okk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int oy = oy_lo + (k >> 1), ox = ox_lo + (k & 1);
          okk[k] = oy <= oy_hi && ox <= ox_hi;
          const size_t o = (o0 + (okk[k] ? (size_t)oy * g.W + ox : 0)) * C + c;
          tq[k] = *reinterpret_cast<const uint2*>(fi.pool_arg + o);
          dq[k] = gld16(Dp + o);
          fq[k] = gld16(Fp + o);
        }
        const uint4 xq = gld16((const T*)fi.v.x + (size_t)pix * C + c);
        float xv[8], d[8];
        {
          float2 af[8];
          affine8_lds(aft + PI * C, c, af);
          unpack_bf8(xq, xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) { xv[j] = fuse_act<ACT>(xv[j], af[j], fi.v.act); d[j] = 0.f; }
        }
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!okk[k]) continue;
          const int oy = oy_lo + (k >> 1), ox = ox_lo + (k & 1);
          const int kme = (iy - (oy * 2 - pt)) * 3 + (ix - (ox * 2 - pl));
          float F[8], dd[8];
          fuse_df<OACT>(dq[k], fq[k], F, dd);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int tap = (int)(((j < 4 ? tq[k].x : tq[k].y) >> (8 * (j & 3))) & 0xffu);
            if (tap == kme) {
              d[j] += dd[j];
              s += dd[j] * (xv[j] - F[j]);
            }
          }
        }
        part[PI] = s;
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] *= wn[PI];
        acc8m((T*)fi.dx + (size_t)pix * C + c, 8, d, fi.accumulate);
      }
    }
  }
  if (PI < 0 || b >= g.nb_pool) {
    const long q = (long)(b - g.nb_pool) * 256 + tid;
    if (q < (long)g.B * g.QH * g.QW * nv) {
      const int cv = (int)(q % nv), c = cv * 8;
      long r = q / nv;
      const int qx = (int)(r % g.QW);
      r /= g.QW;
      const int qy = (int)(r % g.QH), n = (int)(r / g.QH);
      const size_t o0 = (size_t)n * g.H * g.W;
      bool ok[4];
      size_t po[4];  // element offset of the quad's pixel p (invalid ones alias pixel 0)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int y = 2 * qy + (p >> 1), x = 2 * qx + (p & 1);
        ok[p] = y < g.H && x < g.W;
        po[p] = (o0 + (size_t)(ok[p] ? y : 2 * qy) * g.W + (ok[p] ? x : 2 * qx)) * C + c;
      }
      uint4 dq[4], fq[4], sq[3][4], uq[3];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        dq[p] = gld16(Dp + po[p]);
        fq[p] = gld16(Fp + po[p]);
      }
#pragma unroll
      for (int i = 0; i < NIN; ++i) {
        const T* X = (const T*)g.in[i].v.x;
        if (MODE[i] == EDET_MODE_SAME) {
#pragma unroll
          for (int p = 0; p < 4; ++p) sq[i][p] = gld16(X + po[p]);
        } else if (MODE[i] == EDET_MODE_UPSAMPLE) {
          uq[i] = gld16(X + (((size_t)n * g.in[i].H + qy) * g.in[i].W + qx) * C + c);
        }
      }
      float vu[8], du[8];
#pragma unroll
      for (int i = 0; i < NIN; ++i) {
        if (MODE[i] == EDET_MODE_UPSAMPLE) {
          float2 af[8];
          affine8_lds(aft + i * C, c, af);
          unpack_bf8(uq[i], vu);
#pragma unroll
          for (int j = 0; j < 8; ++j) { vu[j] = fuse_act<ACT>(vu[j], af[j], g.in[i].v.act); du[j] = 0.f; }
        }
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (!ok[p]) continue;
        float F[8], d[8];
        fuse_df<OACT>(dq[p], fq[p], F, d);
#pragma unroll
        for (int i = 0; i < NIN; ++i) {
          if (MODE[i] == EDET_MODE_SAME) {
            float2 af[8];
            affine8_lds(aft + i * C, c, af);
            float v[8], o[8], s = 0.f;
            unpack_bf8(sq[i][p], v);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              s += d[j] * (fuse_act<ACT>(v[j], af[j], g.in[i].v.act) - F[j]);
              o[j] = d[j] * wn[i];
            }
            part[i] += s;
            acc8m((T*)g.in[i].dx + po[p], 8, o, g.in[i].accumulate);
          } else if (MODE[i] == EDET_MODE_UPSAMPLE) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              s += d[j] * (vu[j] - F[j]);
              du[j] += d[j];
            }
            part[i] += s;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NIN; ++i) {
        if (MODE[i] == EDET_MODE_UPSAMPLE) {
#pragma unroll
          for (int j = 0; j < 8; ++j) du[j] *= wn[i];
          acc8m((T*)g.in[i].dx + (((size_t)n * g.in[i].H + qy) * g.in[i].W + qx) * C + c, 8, du,
                g.in[i].accumulate);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float s = wave_sum(part[i]);
    if (lane == 0) red[i][wave] = s;
  }
  __syncthreads();
  if (tid == 0) {
    float4 o;
    o.x = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    o.y = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    o.z = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);
    o.w = 0.f;
    g.part[b] = o;
  }
}

// dw[i] += (sum over the node's blocks of part[.][i]) / (sum w + 1e-4), per node; the blocks'
// sums added in a fixed order (fp64), so the result does not depend on scheduling
struct FuseFoldArgs {
  edet_fuse_fold it[EDET_FUSE_FOLD_MAX];
};
__global__ __launch_bounds__(256) void k_fuse_fold(FuseFoldArgs a) {
  __shared__ double red[3][4];
  const edet_fuse_fold f = a.it[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float4* P = (const float4*)f.part;
  double s[3] = {0.0, 0.0, 0.0};
  for (int b = tid; b < f.nparts; b += 256) {
    const float4 p = P[b];
    s[0] += p.x; s[1] += p.y; s[2] += p.z;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double v = s[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[i][wave] = v;
  }
  __syncthreads();
  if (tid < f.n_in) {
    const double t = (red[tid][0] + red[tid][1]) + (red[tid][2] + red[tid][3]);
    f.dw[tid] += (float)(t / (double)fuse_denom(f.w, f.n_in));
  }
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_stem_fwd(int dtype, const void* x, int B, int H, int W, const void* w, int Cout,
                  void* y, double* sum, double* sq, edet_stream_t stream) {
  EDET_REQUIRE(x && w && y && sum && sq, "stem_fwd: null argument");
  EDET_REQUIRE(Cout % 8 == 0 && Cout <= 64, "stem_fwd: Cout must be a multiple of 8, <= 64");
  const long px = (long)B * cdiv(H, 2) * cdiv(W, 2);
  const int nb = (int)((px + 255) / 256);
  if (dtype == EDET_BF16 && Cout % 16 == 0 && px > 0) {
    const int OH = cdiv(H, 2), OW = cdiv(W, 2);
    const int R = std::max(1, std::min(8, 1024 / OW));
    const size_t lds = (size_t)(2 * R + 1) * cdiv(W * 3, 8) * 8 * 2;
    EDET_REQUIRE(lds <= 64 * 1024, "stem_fwd: image rows too wide (W=%d)", W);
    const int grid = B * cdiv(OH, R);
    const uint16_t* xb = (const uint16_t*)x;
    const uint16_t* wb = (const uint16_t*)w;
    uint16_t* yb = (uint16_t*)y;
    hipStream_t st = (hipStream_t)stream;
    switch (Cout / 16) {
      case 1: EDET_LAUNCH(k_stem2_fwd<1>, dim3(grid), dim3(256), lds, st, xb, B, H, W, wb, Cout, yb, sum, sq, R); break;
      case 2: EDET_LAUNCH(k_stem2_fwd<2>, dim3(grid), dim3(256), lds, st, xb, B, H, W, wb, Cout, yb, sum, sq, R); break;
      case 3: EDET_LAUNCH(k_stem2_fwd<3>, dim3(grid), dim3(256), lds, st, xb, B, H, W, wb, Cout, yb, sum, sq, R); break;
      default: EDET_LAUNCH(k_stem2_fwd<4>, dim3(grid), dim3(256), lds, st, xb, B, H, W, wb, Cout, yb, sum, sq, R); break;
    }
    return check_launch("edet stem2_fwd");
  }
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_stem_fwd<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const T*)x, B, H, W,
                               (const T*)w, Cout, (T*)y, sum, sq);
    return check_launch("edet stem_fwd");
  });
}

int edet_stem_wgrad(int dtype, const void* x, int B, int H, int W, const void* dy, int Cout,
                    float* dw, edet_stream_t stream) {
  EDET_REQUIRE(x && dy && dw, "stem_wgrad: null argument");
  EDET_REQUIRE(Cout % 8 == 0 && Cout <= 64, "stem_wgrad: Cout must be a multiple of 8, <= 64");
  const long px = (long)B * cdiv(H, 2) * cdiv(W, 2);
  if (dtype == EDET_BF16 && Cout % 16 == 0 && px > 0) {
    const int OH = cdiv(H, 2), OW = cdiv(W, 2);
    // strips of <= 256 output pixels and 1024 blocks: at 256^2 outputs one row per strip holds the
    // LDS image at 29 KB (5 blocks per CU instead of 2), 120 -> 91 us (r05y sweep).  Development
    // slots 48 / 49: output rows per strip / block cap
    const int R = dev_knob(48) > 0 ? dev_knob(48) : std::max(1, std::min(8, 256 / OW));
    const size_t lds = std::max((size_t)(2 * R + 1) * cdiv(W * 3, 8) * 8 * 2 + (size_t)R * OW * (Cout + 8) * 2,
                                (size_t)4 * 32 * Cout * 4);
    const int grid = std::min(B * cdiv(OH, R), dev_knob(49) > 0 ? dev_knob(49) : 1024);
    float* part = workspace_f32((size_t)grid * 27 * Cout);
    if (part && lds <= 96 * 1024) {
      const uint16_t* xb = (const uint16_t*)x;
      const uint16_t* db = (const uint16_t*)dy;
      hipStream_t st = (hipStream_t)stream;
      switch (Cout / 16) {
        case 1: EDET_LAUNCH(k_stem2_wgrad<1>, dim3(grid), dim3(256), lds, st, xb, B, H, W, db, Cout, part, R); break;
        case 2: EDET_LAUNCH(k_stem2_wgrad<2>, dim3(grid), dim3(256), lds, st, xb, B, H, W, db, Cout, part, R); break;
        case 3: EDET_LAUNCH(k_stem2_wgrad<3>, dim3(grid), dim3(256), lds, st, xb, B, H, W, db, Cout, part, R); break;
        default: EDET_LAUNCH(k_stem2_wgrad<4>, dim3(grid), dim3(256), lds, st, xb, B, H, W, db, Cout, part, R); break;
      }
      int rc = check_launch("edet stem2_wgrad");
      if (rc) return rc;
      return sum_partials(part, grid, 27L * Cout, dw, st);
    }
  }
  long per = (px + 2047) / 2048;  // latency-bound: 512 blocks measured 1.4x slower
  per = ((per + 63) / 64) * 64;
  if (per < 64) per = 64;
  const int nb = (int)((px + per - 1) / per);
  float* part = nullptr;  // 27*Cout weights over 2048 blocks: atomics measured faster
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_stem_wgrad<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, (const T*)x, B, H, W,
                               (const T*)dy, Cout, dw, per, part);
    int rc = check_launch("edet stem_wgrad");
    if (rc || !part || !nb) return rc;
    return sum_partials(part, nb, 27L * Cout, dw, (hipStream_t)stream);
  });
}

int edet_maxpool_fwd(int dtype, const edet_lazy* x, int B, int H, int W, int C, void* y,
                     edet_stream_t stream) {
  EDET_REQUIRE(x && x->x && y, "maxpool_fwd: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0 && x->gate == nullptr, "maxpool_fwd: need C%%8==0, no gate");
  const long n = (long)B * cdiv(H, 2) * cdiv(W, 2) * (C / 8);
  const int nb = (int)((n + 255) / 256);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb)
      EDET_LAUNCH(k_maxpool_fwd<T>, dim3(nb), dim3(256), C * sizeof(float2), (hipStream_t)stream, *x, B, H, W, C, (T*)y,
                  (uint8_t*)nullptr);
    return check_launch("edet maxpool_fwd");
  });
}

int edet_maxpool_fwd_taps(int dtype, const edet_lazy* x, int B, int H, int W, int C, void* y, uint8_t* taps,
                          edet_stream_t stream) {
  EDET_REQUIRE(x && x->x && y && taps, "maxpool_fwd_taps: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0 && x->gate == nullptr, "maxpool_fwd_taps: need C%%8==0, no gate");
  const long n = (long)B * cdiv(H, 2) * cdiv(W, 2) * (C / 8);
  const int nb = (int)((n + 255) / 256);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb)
      EDET_LAUNCH(k_maxpool_fwd<T>, dim3(nb), dim3(256), C * sizeof(float2), (hipStream_t)stream, *x, B, H, W, C, (T*)y,
                  taps);
    return check_launch("edet maxpool_fwd_taps");
  });
}

int edet_maxpool_bwd_taps(int dtype, int B, int H, int W, int C, const uint8_t* taps, const void* dy, void* dx,
                          int accumulate, edet_stream_t stream) {
  EDET_REQUIRE(taps && dy && dx, "maxpool_bwd_taps: null argument");
  EDET_REQUIRE(C % 8 == 0 && B > 0 && H > 0 && W > 0, "maxpool_bwd_taps: need C%%8==0 and a non-empty plane");
  const long n = (long)B * H * W * (C / 8);
  const int nb = (int)((n + 255) / 256);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb)
      EDET_LAUNCH(k_maxpool_bwd_taps<T>, dim3(nb), dim3(256), 0, (hipStream_t)stream, B, H, W, C, taps, (const T*)dy,
                  (T*)dx, accumulate);
    return check_launch("edet maxpool_bwd_taps");
  });
}

int edet_maxpool_bwd(int dtype, const edet_lazy* x, int B, int H, int W, int C,
                     const void* dy, void* dx, int accumulate, edet_stream_t stream) {
  EDET_REQUIRE(x && x->x && dy && dx, "maxpool_bwd: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0 && x->gate == nullptr, "maxpool_bwd: need C%%8==0, no gate");
  const long n = (long)B * H * W * (C / 8);
  const int nb = (int)((n + 255) / 256);
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_maxpool_bwd<T>, dim3(nb), dim3(256), C * sizeof(float2), (hipStream_t)stream, *x, B, H, W, C,
                               (const T*)dy, (T*)dx, accumulate);
    return check_launch("edet maxpool_bwd");
  });
}

static int fuse_setup(FuseArgs& g, int n_in, const edet_fuse_input* ins, const float* w, int B, int H, int W,
                      int C) {
  EDET_REQUIRE(ins && w && n_in >= 1 && n_in <= 3, "bifpn_fuse: 1..3 inputs required");
  EDET_REQUIRE(C % 8 == 0, "bifpn_fuse: need C%%8==0");
  for (int i = 0; i < n_in; ++i) {
    const edet_fuse_input& f = ins[i];
    EDET_REQUIRE(f.v.x && f.v.ld == C && f.v.gate == nullptr, "bifpn_fuse: input %d must be [rows][C]", i);
    if (f.mode == EDET_MODE_SAME)
      EDET_REQUIRE(f.H == H && f.W == W, "bifpn_fuse: input %d size mismatch", i);
    else if (f.mode == EDET_MODE_MAXPOOL)
      EDET_REQUIRE(cdiv(f.H, 2) == H && cdiv(f.W, 2) == W, "bifpn_fuse: input %d pool size mismatch", i);
    else
      EDET_REQUIRE(f.mode == EDET_MODE_UPSAMPLE && f.H > 0 && f.W > 0, "bifpn_fuse: input %d bad mode", i);
    g.in[i] = f;
  }
  g.w = w; g.n_in = n_in; g.B = B; g.H = H; g.W = W; g.C = C;
  return EDET_OK;
}

// the activation every input shares (0 none, 1 swish), -1 if they differ
static int fuse_common_act(int n_in, const edet_fuse_input* ins) {
  const int a = ins[0].v.act ? 1 : 0;
  for (int i = 1; i < n_in; ++i)
    if ((ins[i].v.act ? 1 : 0) != a) return -1;
  return a;
}

int edet_bifpn_fuse_fwd(int dtype, int n_in, const edet_fuse_input* ins, const float* w,
                        int B, int H, int W, int C, void* out, edet_stream_t stream) {
  FuseArgs g{};
  int rc = fuse_setup(g, n_in, ins, w, B, H, W, C);
  if (rc) return rc;
  EDET_REQUIRE(out, "bifpn_fuse_fwd: null out");
  g.out = out;
  const long n = (long)B * H * W * (C / 8);
  int nb = (int)((n + 255) / 256);
  // at most 2048 blocks striding over the vectors, so each block's affine tables serve more
  // than 32 pixels (D4 1605 -> 1401 us, D0 282 -> 271 us per step; profiles/r03ah_fuse_grid.txt).
  // Development slot 28 overrides the cap.
  const int cap = dev_knob(28) > 0 ? dev_knob(28) : 2048;
  if (nb > cap) nb = cap;
  // the BiFPN's input-mode combinations as compile-time forms (bf16; development slot 34 = 2:
  // the runtime-mode kernel)
  if (dtype == EDET_BF16 && nb && dev_knob(34) != 2) {
    const size_t lds = n_in * C * sizeof(float2);
    const int m0 = ins[0].mode, m1 = ins[1].mode, m2 = n_in == 3 ? ins[2].mode : -1;
    constexpr int S_ = EDET_MODE_SAME, U_ = EDET_MODE_UPSAMPLE, P_ = EDET_MODE_MAXPOOL;
    hipStream_t st = (hipStream_t)stream;
    bool hit = true;
    const int act = fuse_common_act(n_in, ins);
#define EDET_FUSE_M(A, B, C)                                                                              \
  do {                                                                                                    \
    if (act == 0) EDET_LAUNCH((k_fuse_fwd_m<A, B, C, 0>), dim3(nb), dim3(256), lds, st, g);                  \
    else if (act == 1) EDET_LAUNCH((k_fuse_fwd_m<A, B, C, 1>), dim3(nb), dim3(256), lds, st, g);             \
    else EDET_LAUNCH((k_fuse_fwd_m<A, B, C, -1>), dim3(nb), dim3(256), lds, st, g);                          \
  } while (0)
    if (m0 == S_ && m1 == U_ && m2 == -1) EDET_FUSE_M(S_, U_, -1);
    else if (m0 == S_ && m1 == S_ && m2 == P_) EDET_FUSE_M(S_, S_, P_);
    else if (m0 == S_ && m1 == P_ && m2 == -1) EDET_FUSE_M(S_, P_, -1);
    else if (m0 == S_ && m1 == S_ && m2 == U_) EDET_FUSE_M(S_, S_, U_);
    else if (m0 == S_ && m1 == S_ && m2 == -1) EDET_FUSE_M(S_, S_, -1);
    else hit = false;
#undef EDET_FUSE_M
    if (hit) return check_launch("edet bifpn_fuse_fwd");
  }
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_fuse_fwd<T>, dim3(nb), dim3(256), n_in * C * sizeof(float2), (hipStream_t)stream, g);
    return check_launch("edet bifpn_fuse_fwd");
  });
}

int edet_bifpn_fuse_bwd(int dtype, int n_in, const edet_fuse_input* ins, const float* w,
                        int B, int H, int W, int C, const void* out, const void* dout,
                        float* dw, edet_stream_t stream) {
  FuseArgs g{};
  int rc = fuse_setup(g, n_in, ins, w, B, H, W, C);
  if (rc) return rc;
  EDET_REQUIRE(out && dout && dw, "bifpn_fuse_bwd: null argument");
  for (int i = 0; i < n_in; ++i) EDET_REQUIRE(ins[i].dx, "bifpn_fuse_bwd: input %d has no dx", i);
  g.fused = out; g.dout = dout; g.dw = dw;
  g.nb_w = (int)std::min<long>(256, ((long)B * H * W * (C / 8) + 255) / 256);
  int nb = g.nb_w;
  for (int i = 0; i < n_in; ++i) {
    g.nb_in[i] = (int)(((long)B * ins[i].H * ins[i].W * (C / 8) + 255) / 256);
    nb += g.nb_in[i];
  }
  if (dtype == EDET_BF16 && nb && dev_knob(34) != 2) {
    const size_t lds = n_in * C * sizeof(float2);
    const int m0 = ins[0].mode, m1 = ins[1].mode, m2 = n_in == 3 ? ins[2].mode : -1;
    constexpr int S_ = EDET_MODE_SAME, U_ = EDET_MODE_UPSAMPLE, P_ = EDET_MODE_MAXPOOL;
    hipStream_t st = (hipStream_t)stream;
    bool hit = true;
    const int act = fuse_common_act(n_in, ins);
#define EDET_FUSE_M(A, B, C)                                                                              \
  do {                                                                                                    \
    if (act == 0) EDET_LAUNCH((k_fuse_bwd_m<A, B, C, 0>), dim3(nb), dim3(256), lds, st, g);                  \
    else if (act == 1) EDET_LAUNCH((k_fuse_bwd_m<A, B, C, 1>), dim3(nb), dim3(256), lds, st, g);             \
    else EDET_LAUNCH((k_fuse_bwd_m<A, B, C, -1>), dim3(nb), dim3(256), lds, st, g);                          \
  } while (0)
    if (m0 == S_ && m1 == U_ && m2 == -1) EDET_FUSE_M(S_, U_, -1);
    else if (m0 == S_ && m1 == S_ && m2 == P_) EDET_FUSE_M(S_, S_, P_);
    else if (m0 == S_ && m1 == P_ && m2 == -1) EDET_FUSE_M(S_, P_, -1);
    else if (m0 == S_ && m1 == S_ && m2 == U_) EDET_FUSE_M(S_, S_, U_);
    else if (m0 == S_ && m1 == S_ && m2 == -1) EDET_FUSE_M(S_, S_, -1);
    else hit = false;
#undef EDET_FUSE_M
    if (hit) return check_launch("edet bifpn_fuse_bwd");
  }
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (nb) EDET_LAUNCH(k_fuse_bwd<T>, dim3(nb), dim3(256), n_in * C * sizeof(float2), (hipStream_t)stream, g);
    return check_launch("edet bifpn_fuse_bwd");
  });
}

// the one-pass backward's plan: 0 blocks = this node is not covered (dtype, input-mode
// combination, an upsample that is not exactly x2, a max-pooled input without recorded taps)
static long fuse_dv_plan(int dtype, int n_in, const edet_fuse_input* ins, int B, int H, int W, int C,
                         int* nb_pool) {
  *nb_pool = 0;
  if (dtype != EDET_BF16 || n_in < 2 || n_in > 3 || C % 8 || dev_knob(34) == 2) return 0;
  const int m0 = ins[0].mode, m1 = ins[1].mode, m2 = n_in == 3 ? ins[2].mode : -1;
  constexpr int S_ = EDET_MODE_SAME, U_ = EDET_MODE_UPSAMPLE, P_ = EDET_MODE_MAXPOOL;
  const bool combo = (m0 == S_ && m1 == U_ && m2 == -1) || (m0 == S_ && m1 == S_ && m2 == P_) ||
                     (m0 == S_ && m1 == P_ && m2 == -1) || (m0 == S_ && m1 == S_ && m2 == U_) ||
                     (m0 == S_ && m1 == S_ && m2 == -1);
  if (!combo) return 0;
  const int nv = C / 8;
  for (int i = 0; i < n_in; ++i) {
    const edet_fuse_input& f = ins[i];
    if (f.mode == U_ && (H != 2 * f.H || W != 2 * f.W)) return 0;
    if (f.mode == P_) {
      if (!f.pool_arg) return 0;
      *nb_pool = (int)(((long)B * f.H * f.W * nv + 255) / 256);
    }
  }
  return *nb_pool + ((long)B * cdiv(H, 2) * cdiv(W, 2) * nv + 255) / 256;
}

int edet_bifpn_fuse_bwd_dv_parts(int dtype, int n_in, const edet_fuse_input* ins, int B, int H, int W, int C,
                                 int* nparts) {
  EDET_REQUIRE(nparts && (n_in == 0 || ins), "bifpn_fuse_bwd_dv_parts: null argument");
  int nbp;
  const long nb = fuse_dv_plan(dtype, n_in, ins, B, H, W, C, &nbp);
  EDET_REQUIRE(nb < (1L << 31), "bifpn_fuse_bwd_dv_parts: too many blocks");
  *nparts = (int)nb;
  return EDET_OK;
}

int edet_bifpn_fuse_bwd_dv(int dtype, int n_in, const edet_fuse_input* ins, const float* w, int B, int H, int W,
                           int C, const void* out, const void* dv, int out_act, float* part, int nparts,
                           edet_stream_t stream) {
  FuseDvArgs g{};
  FuseArgs s{};
  int rc = fuse_setup(s, n_in, ins, w, B, H, W, C);
  if (rc) return rc;
  EDET_REQUIRE(out && dv && part, "bifpn_fuse_bwd_dv: null argument");
  EDET_REQUIRE(out_act == 0 || out_act == 1, "bifpn_fuse_bwd_dv: out_act must be 0 or 1");
  for (int i = 0; i < n_in; ++i) EDET_REQUIRE(ins[i].dx, "bifpn_fuse_bwd_dv: input %d has no dx", i);
  int nbp;
  const long nb = fuse_dv_plan(dtype, n_in, ins, B, H, W, C, &nbp);
  EDET_REQUIRE(nb > 0, "bifpn_fuse_bwd_dv: node not covered (edet_bifpn_fuse_bwd_dv_parts returned 0)");
  EDET_REQUIRE(nparts == nb, "bifpn_fuse_bwd_dv: nparts %d, the plan has %ld", nparts, nb);
  for (int i = 0; i < n_in; ++i) g.in[i] = ins[i];
  g.w = w; g.fused = out; g.dv = dv; g.part = (float4*)part;
  g.B = B; g.H = H; g.W = W; g.C = C; g.QH = cdiv(H, 2); g.QW = cdiv(W, 2);
  g.nb_pool = nbp;
  const size_t lds = n_in * C * sizeof(float2);
  const int m0 = ins[0].mode, m1 = ins[1].mode, m2 = n_in == 3 ? ins[2].mode : -1;
  constexpr int S_ = EDET_MODE_SAME, U_ = EDET_MODE_UPSAMPLE, P_ = EDET_MODE_MAXPOOL;
  hipStream_t st = (hipStream_t)stream;
  const int act = fuse_common_act(n_in, ins);
#define EDET_FUSE_DV(A, B_, C_, OA)                                                                       \
  do {                                                                                                   \
    if (act == 0) EDET_LAUNCH((k_fuse_bwd_dv<A, B_, C_, 0, OA>), dim3(nb), dim3(256), lds, st, g);       \
    else if (act == 1) EDET_LAUNCH((k_fuse_bwd_dv<A, B_, C_, 1, OA>), dim3(nb), dim3(256), lds, st, g);  \
    else EDET_LAUNCH((k_fuse_bwd_dv<A, B_, C_, -1, OA>), dim3(nb), dim3(256), lds, st, g);               \
  } while (0)
#define EDET_FUSE_DV2(A, B_, C_)                   \
  do {                                             \
    if (out_act) EDET_FUSE_DV(A, B_, C_, 1);       \
    else EDET_FUSE_DV(A, B_, C_, 0);               \
  } while (0)
  if (m0 == S_ && m1 == U_ && m2 == -1) EDET_FUSE_DV2(S_, U_, -1);
  else if (m0 == S_ && m1 == S_ && m2 == P_) EDET_FUSE_DV2(S_, S_, P_);
  else if (m0 == S_ && m1 == P_ && m2 == -1) EDET_FUSE_DV2(S_, P_, -1);
  else if (m0 == S_ && m1 == S_ && m2 == U_) EDET_FUSE_DV2(S_, S_, U_);
  else EDET_FUSE_DV2(S_, S_, -1);
#undef EDET_FUSE_DV2
#undef EDET_FUSE_DV
  return check_launch("edet bifpn_fuse_bwd_dv");
}

int edet_bifpn_fuse_fold(int n, const edet_fuse_fold* items, edet_stream_t stream) {
  EDET_REQUIRE(n >= 0 && (n == 0 || items), "bifpn_fuse_fold: bad arguments");
  for (int i = 0; i < n; ++i)
    EDET_REQUIRE(items[i].part && items[i].w && items[i].dw && items[i].nparts >= 0 && items[i].n_in >= 1 &&
                     items[i].n_in <= 3,
                 "bifpn_fuse_fold: bad item %d", i);
  for (int i0 = 0; i0 < n; i0 += EDET_FUSE_FOLD_MAX) {
    const int m = std::min(n - i0, EDET_FUSE_FOLD_MAX);
    FuseFoldArgs a{};
    for (int i = 0; i < m; ++i) a.it[i] = items[i0 + i];
    EDET_LAUNCH(k_fuse_fold, dim3(m), dim3(256), 0, (hipStream_t)stream, a);
  }
  return check_launch("edet bifpn_fuse_fold");
}

}  // extern "C"
