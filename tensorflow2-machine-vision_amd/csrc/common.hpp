// Shared device helpers for libedet (gfx950 / CDNA4).
//
// Storage types: float (EDET_F32) or bf16 held as uint16_t (EDET_BF16). All arithmetic is
// fp32. Activations are NHWC rows ([rows][ld]); 8-element vectors are the unit of global
// access (16 B for bf16, 32 B for fp32) so every row stride handed to a vector path must be
// a multiple of 8 elements.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/edet.h"

namespace edet {

// ------------------------------------------------------------------ error reporting
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// measurement: remember the kernel each launch site starts (edet_launched_kernels)
void note_kernel(const char* site);
#define EDET_LAUNCH(K, ...)                 \
  do {                                      \
    ::edet::note_kernel(#K);                \
    hipLaunchKernelGGL(K, __VA_ARGS__);     \
  } while (0)
// Development A/B slots (edet_dev_set): plan overrides for scripts/kbench.py --dev, compiled
// only into the EDET_DEV build (`make dev` -> lib/libedet_dev.so).  The production library
// folds every slot to 0 (the measured plans) and its edet_dev_set returns EDET_EUNSUPPORTED.
#ifdef EDET_DEV
int dev_knob(int slot);
#else
constexpr int dev_knob(int) { return 0; }
#endif
// registered scratch (edet_set_workspace) if it holds n floats, else nullptr
float* workspace_f32(size_t n_floats);
// out[i] += sum_s part[s*n + i], fixed order
// out[i] += sum_s part[s][i] (i < n), and out2[j] += sum_s part[S * n + s * n2 + j] (j < n2) in
// the same launch when out2 is non-null
int sum_partials(const float* part, int S, long n, float* out, hipStream_t st, long n2 = 0, float* out2 = nullptr);

#define EDET_REQUIRE(cond, ...)            \
  do {                                     \
    if (!(cond)) {                         \
      ::edet::set_error(__VA_ARGS__);      \
      return EDET_EINVAL;                  \
    }                                      \
  } while (0)

// ------------------------------------------------------------------ vector types
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving
  return __builtin_bit_cast(uint16_t, h);
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<uint16_t>(uint16_t v) { return bf2f(v); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t from_f<uint16_t>(float v) { return f2bf(v); }

// 8 contiguous elements -> fp32 (pointer 16-B aligned)
__device__ __forceinline__ void ld8(const float* p, float* o) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void ld8(const uint16_t* p, float* o) {
  uint4 v = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void st8(uint16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
// masked variants: elements [0, n) valid, others read as 0 / not written
template <typename T>
__device__ __forceinline__ void ld8m(const T* p, int n, float* o) {
  if (n >= 8) { ld8(p, o); return; }
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (i < n) ? to_f<T>(p[i]) : 0.f;
}
template <typename T>
__device__ __forceinline__ void st8m(T* p, int n, const float* v) {
  if (n >= 8) { st8(p, v); return; }
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < n) p[i] = from_f<T>(v[i]);
}
// read-modify-write accumulate of 8 elements
template <typename T>
__device__ __forceinline__ void acc8m(T* p, int n, const float* v, int accumulate) {
  float o[8];
  if (accumulate) {
    ld8m(p, n, o);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] += v[i];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = v[i];
  }
  st8m(p, n, o);
}

// ------------------------------------------------------------------ math
// v_rcp_f32 (1 ulp) instead of the correctly rounded division the build flags select for
// '/': the swish of every lazy load runs through here (-4 % step time measured)
__device__ __forceinline__ float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float swishf_(float x) { return x * sigmoidf_(x); }
__device__ __forceinline__ float dswishf_(float x) {
  float s = sigmoidf_(x);
  return s * (1.f + x * (1.f - s));
}

// fp64 statistics accumulation (one atomic per channel per block; DESIGN.md "Reproducibility")
__device__ __forceinline__ void stat_add(double* p, double v) { atomicAdd(p, v); }

// Replicated per-channel statistics (ABI 9; include/edet.h "statistics vectors").  Every block
// of a producer adds its per-channel sums into the same fp64 vector; the adds to one address
// serialise at the memory-side atomic unit (~20 ns each: 256 adders cost ~5 us per launch, the
// D0 step ~0.5 ms; r06e/r06g).  The BN batch statistics and the BN-backward sums are therefore
// kept in EDET_STAT_REPLICAS = 4 replicas: channel c, replica r at stat_idx(c, r) -- 16
// channels of one replica per 128-B line, so replicas never share a line -- a block adds into
// the replica its index hashes to, and readers take the value as the fixed-order sum of the
// four.  A vector of C channels occupies stat_len(C) doubles.
constexpr int SR = EDET_STAT_REPLICAS;
static_assert(SR == 4, "stat_get sums four replicas");
__host__ __device__ __forceinline__ constexpr long stat_len(int C) { return (long)((C + 15) / 16) * 16 * SR; }
__host__ __device__ __forceinline__ int stat_idx(int c, int r) { return (c >> 4) * (16 * SR) + r * 16 + (c & 15); }
__device__ __forceinline__ double stat_get(const double* p, int c) {
  const double* q = p + stat_idx(c, 0);
  return (q[0] + q[16]) + (q[32] + q[48]);
}
// a block's replica: a multiplicative hash of its index (grids whose blocks of one channel group
// are a fixed stride apart, e.g. the depthwise channel blocks, still spread over all four)
__device__ __forceinline__ int stat_rep() { return (int)((blockIdx.x * 2654435761u) >> 30); }
__device__ __forceinline__ void stat_put(double* p, int c, double v) { atomicAdd(p + stat_idx(c, stat_rep()), v); }

// Sum over the four 16-lane rows of a wave (lane bits 4 and 5), result in every lane: the
// MFMA epilogues reduce a column's 4 row groups this way.  gfx950's v_permlane16/32_swap are
// plain VALU ops; the __shfl_xor form was two dependent ds_bpermute round trips per value
// (the BN-statistics epilogue cost 25 us of a 90 us GEMM).  Same additions, same order.
__device__ __forceinline__ float row4_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Sum over the 16 lanes of a DPP row (lane bits 0-3), result in every lane: four DPP adds
// (plain VALU) instead of four __shfl_xor rounds, each a ds_bpermute LDS round trip (the
// k_gemm_s statistics flush meets a new pyramid level about once per row group: its
// shuffles cost more than the group's MFMAs)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2 (each lane: its quad's sum)
  v += dpp_f<0x141>(v);  // row_half_mirror: the other quad of the 8-lane half
  v += dpp_f<0x140>(v);  // row_mirror: the other half of the row
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }
// floor division for possibly negative numerators (b > 0)
__device__ __forceinline__ int fdiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// TF 'SAME' padding: returns pad_before; out = ceil(in / s)
__host__ __device__ __forceinline__ int same_pad(int in, int k, int s) {
  int out = (in + s - 1) / s;
  int tot = (out - 1) * s + k - in;
  if (tot < 0) tot = 0;
  return tot / 2;
}

// ------------------------------------------------------------------ pyramid helpers
__host__ __device__ __forceinline__ int seg_rows(const edet_pyramid& p, int s) {
  return p.batch * p.H[s] * p.W[s];
}
__host__ __device__ __forceinline__ int seg_of_row(const edet_pyramid& p, int row) {
  int s = 0;
  for (int i = 1; i < p.nseg; ++i)
    if (row >= p.row_off[i]) s = i;
  return s;
}
// Range-checked 16-byte loads (buffer_load_dwordx4 through a descriptor over [base, base +
// bytes)): an offset at or past the range reads zeros.  A pipelined loop fetches its operand
// tiles with these -- the bounds are in the offset, the load itself is unconditional and its
// result needs no select -- so the compiler's wait before a commit counts just that stage's
// loads (loads under branches, or selected after, left it waiting for every stage in flight).
// The descriptor must come from wave-uniform values; callers pass kernel-argument pointers
// advanced by block-uniform amounts.
constexpr uint32_t BUF_OOB = 0x80000000u;
// a load the compiler knows is global (a pointer it cannot place becomes a flat load, which the
// wait-count pass orders against LDS and every load in flight)
__device__ __forceinline__ float gld(const float* p) {
  return *(const __attribute__((address_space(1))) float*)p;
}
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gld16(const void* p) {
  const u32x4_t v = *(const __attribute__((address_space(1))) u32x4_t*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, long bytes) {
  const uint32_t n = bytes <= 0 ? 0u : (bytes >= (long)BUF_OOB ? BUF_OOB : (uint32_t)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}
// off when ok, else an offset past any range -- as arithmetic: a select here was turned into
// control flow around the load, and the register merge after it cost a full wait
__device__ __forceinline__ uint32_t buf_off(bool ok, uint32_t off) { return off | ((uint32_t)!ok << 31); }
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// seg_of_row for a per-lane row, plus the end of that segment's valid rows: compile-time
// segment indices only, so the pyramid stays in scalar registers (a per-lane index into the
// kernel-argument struct becomes per-lane vector loads, each waited for at once -- with the
// in-order vmcnt counter, behind every load already in flight)
__device__ __forceinline__ int seg_of_row_end(const edet_pyramid& p, int row, int& end) {
  int s = 0, e = p.row_off[0] + seg_rows(p, 0);
#pragma unroll
  for (int i = 1; i < EDET_MAX_SEG; ++i) {
    const bool in = i < p.nseg && row >= p.row_off[i];
    s = in ? i : s;
    e = in ? p.row_off[i] + seg_rows(p, i) : e;
  }
  end = e;
  return s;
}
__host__ __device__ __forceinline__ int pyr_valid_rows(const edet_pyramid& p) {
  int n = 0;
  for (int i = 0; i < p.nseg; ++i) n += seg_rows(p, i);
  return n;
}
__host__ __device__ __forceinline__ int pyr_total_rows(const edet_pyramid& p) {
  return p.row_off[p.nseg - 1] + seg_rows(p, p.nseg - 1);
}

// Per-channel affine of the lazy BN for segment `seg`: v = x * sc + sh.
__device__ __forceinline__ float2 bn_affine(const edet_bn& bn, int seg, int c, float inv_count) {
  if (!bn.enabled) return make_float2(1.f, 0.f);
  const double mean = stat_get(bn.sum[seg], c) * (double)inv_count;
  const double var = fmax(stat_get(bn.sq[seg], c) * (double)inv_count - mean * mean, 0.0);
  const float r = rsqrtf((float)var + bn.eps);
  const float sc = bn.gamma[seg][c] * r;
  return make_float2(sc, bn.beta[seg][c] - (float)mean * sc);
}
// mean / rstd (for x-hat in backward)
__device__ __forceinline__ float2 bn_mean_rstd(const edet_bn& bn, int seg, int c, float inv_count) {
  const double mean = stat_get(bn.sum[seg], c) * (double)inv_count;
  const double var = fmax(stat_get(bn.sq[seg], c) * (double)inv_count - mean * mean, 0.0);
  return make_float2((float)mean, rsqrtf((float)var + bn.eps));
}

__device__ __forceinline__ float lazy_apply(float x, float2 af, int act) {
  float v = x * af.x + af.y;
  return act ? swishf_(v) : v;
}

// Bijective XCD-aware block remap: blocks b and b+8 share an XCD (round-robin dispatch),
// so give each XCD a contiguous range of logical tile ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Segment-chunked row iteration: each segment is split into chunks of CH rows so a chunk
// never straddles segments.  Returns (seg, chunk-in-seg) for a linear chunk id.
__host__ __device__ __forceinline__ int total_chunks(const edet_pyramid& p, int CH) {
  int t = 0;
  for (int s = 0; s < p.nseg; ++s) t += cdiv(seg_rows(p, s), CH);
  return t;
}
__device__ __forceinline__ void chunk_lookup(const edet_pyramid& p, int CH, int id, int& seg, int& chunk) {
  for (int s = 0; s < p.nseg; ++s) {
    int n = cdiv(seg_rows(p, s), CH);
    if (id < n) { seg = s; chunk = id; return; }
    id -= n;
  }
  seg = p.nseg - 1; chunk = id;  // unreachable with a correct grid
}

}  // namespace edet

#define EDET_DTYPE_DISPATCH(dtype, T, ...)                 \
  do {                                                     \
    if ((dtype) == EDET_F32) {                             \
      using T = float;                                     \
      __VA_ARGS__;                                         \
    } else if ((dtype) == EDET_BF16) {                     \
      using T = uint16_t;                                  \
      __VA_ARGS__;                                         \
    } else {                                               \
      ::edet::set_error("unsupported dtype %d", (dtype));  \
      return EDET_EUNSUPPORTED;                            \
    }                                                      \
  } while (0)
