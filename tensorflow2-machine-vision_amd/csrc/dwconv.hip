// Depthwise k x k convolution, stride 1/2, TF 'SAME' padding (pad_before = floor(total/2),
// the extra row/column at the bottom/right), NHWC, over single tensors or the P3..P7 pyramid.
//
// Replaces DepthwiseConv2D in layers/mb_conv_block.py:85-91,147 and the depthwise half of
// SeparableConv2D in layers/bifpn.py:16-21, layers/class_net.py:46-76, layers/box_net.py:49-78.
//
// Work unit: one workgroup = one image x one 8x8 output tile x 32 channels.  The input halo
// tile ((8-1)*s + k)^2 x 32 is staged once into LDS as fp32 with the lazy BN/swish/SE-gate
// transform of the producer applied on the way in (zero outside the image, i.e. the padding
// is applied to the *transformed* value exactly as the reference pads the layer input).
// Thread (c, r) then produces the 8 outputs of row r for channel c.  The epilogue reduces the
// per-channel BN statistics of the output.
#include "common.hpp"

namespace edet {

constexpr int DTS = 8;   // spatial tile
constexpr int DCB = 32;  // channels per block

struct DwArgs {
  const void* x;
  const void* w;
  void* y;
  const void* dy;
  void* dx;
  float* dw;
  edet_lazy lz;
  edet_pyramid pin, pout;
  edet_statout stats;
  int C, ncb, accumulate, has_stats;
  int tiles_per_wg, tiles_total;
  float* part;  // wgrad: per-chunk partials [chunks][K*K][C] (null: atomics)
  edet_lazy yv;  // fwd + squeeze: the output's own lazy transform (inference BN, act)
  double* sq;    // fwd + squeeze: [batch][C] += mean_hw v(y)  (null: no squeeze)
  edet_dgrad_lazy dyl;  // bwd with a lazy dy (k_dwt GIN): dy = d(raw y) built on load
};

// The N filter taps of channel ch (stride C between taps) into fp32 registers.  Every load is
// issued unconditionally from a clamped channel and zeroed after: a select-predicated load is
// compiled as a branch around it with its own vmcnt(0), i.e. N serial L2 round trips in every
// block's prologue (25 at k5).
template <int N, typename T>
__device__ __forceinline__ void load_taps(float (&wr)[N], const T* w, int C, int ch, bool valid) {
  const T* p = w + (valid ? ch : 0);
  T raw[N];
#pragma unroll
  for (int i = 0; i < N; ++i) raw[i] = p[(size_t)i * C];
#pragma unroll
  for (int i = 0; i < N; ++i) wr[i] = valid ? to_f<T>(raw[i]) : 0.f;
}

// tiles over a pyramid's spatial extent (per channel block)
__device__ __forceinline__ void locate_tile(const edet_pyramid& p, int id, int& seg, int& n, int& ty, int& tx) {
  seg = 0;
  for (; seg < p.nseg - 1; ++seg) {
    const int cnt = p.batch * cdiv(p.H[seg], DTS) * cdiv(p.W[seg], DTS);
    if (id < cnt) break;
    id -= cnt;
  }
  const int ntx = cdiv(p.W[seg], DTS), nty = cdiv(p.H[seg], DTS);
  tx = id % ntx; id /= ntx;
  ty = id % nty;
  n = id / nty;
}
static int host_tiles(const edet_pyramid& p) {
  int t = 0;
  for (int s = 0; s < p.nseg; ++s) t += p.batch * cdiv(p.H[s], DTS) * cdiv(p.W[s], DTS);
  return t;
}

// Stage the transformed input halo of one tile into LDS (fp32, [IH][IW][DCB]) in two halves so
// the loads are all in flight together: fetch issues every raw vector of the tile into
// registers with select-predicated addresses (a load wrapped in a divergent `if` is waited on
// inside it, one latency per vector), commit transforms them into LDS once the tile's affine
// and gate are in LDS.
template <typename T, int IH, int IW>
struct Stage {
  static constexpr int NV = (IH * IW * (DCB / 8) + 255) / 256;
  static constexpr int WORDS = sizeof(T) == 2 ? 1 : 2;
  uint4 raw[NV][WORDS];
  uint32_t ok;
  __device__ __forceinline__ void fetch(const DwArgs& g, int seg, int n, int iy0, int ix0, int c0) {
    const int H = g.pin.H[seg], W = g.pin.W[seg];
    const T* X = (const T*)g.x + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * g.lz.ld + c0;
    ok = 0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = threadIdx.x + u * 256;
      const int pix = v >> 2, cv = (v & 3) * 8;
      const int yy = pix / IW, xx = pix - yy * IW;
      const int gy = iy0 + yy, gx = ix0 + xx;
      const bool in = v < IH * IW * 4 && gy >= 0 && gy < H && gx >= 0 && gx < W && c0 + cv < g.C;
      const uint4* src = reinterpret_cast<const uint4*>(X + (in ? (uint32_t)(gy * W + gx) * g.lz.ld + cv : 0u));
      raw[u][0] = src[0];
      if constexpr (WORDS == 2) raw[u][1] = src[1];
      ok |= (uint32_t)in << u;
    }
  }
  __device__ __forceinline__ void commit(const DwArgs& g, float* tile, const float2* xf, const float* gt) const {
    // a thread's 8 channels are the same for every u (256 % 4 == 0): their affine and gate in
    // registers once (read per element, the tile stores made the compiler reload them)
    const int cv0 = (threadIdx.x & 3) * 8;
    float2 a8[8];
    float g8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a8[j] = xf[cv0 + j]; g8[j] = gt[cv0 + j]; }
    const int act = g.lz.act;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = threadIdx.x + u * 256;
      if (v >= IH * IW * 4) break;
      const int pix = v >> 2, cv = (v & 3) * 8;
      float vals[8];
      if constexpr (WORDS == 1) {
        const uint32_t w4[4] = {raw[u][0].x, raw[u][0].y, raw[u][0].z, raw[u][0].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          vals[2 * i] = __uint_as_float(w4[i] << 16);
          vals[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
        }
      } else {
        const uint32_t w8[8] = {raw[u][0].x, raw[u][0].y, raw[u][0].z, raw[u][0].w,
                                raw[u][1].x, raw[u][1].y, raw[u][1].z, raw[u][1].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) vals[i] = __uint_as_float(w8[i]);
      }
      const bool in = (ok >> u) & 1;
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = in ? lazy_apply(vals[j], a8[j], act) * g8[j] : 0.f;
      float* d = tile + pix * DCB + cv;
      reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
      reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
    }
  }
};

__device__ __forceinline__ void prep_xf(const DwArgs& g, float2* xf, float* gt, int seg, int n, int c0) {
  const int tid = threadIdx.x;
  if (tid < DCB) {
    const int cc = c0 + tid;
    float2 af = make_float2(1.f, 0.f);
    float gv = 1.f;
    if (cc < g.C) {
      af = bn_affine(g.lz.bn, seg, cc, 1.f / (float)seg_rows(g.pin, seg));
      if (g.lz.gate) gv = g.lz.gate[(size_t)n * g.C + cc];
    }
    xf[tid] = af;
    gt[tid] = gv;
  }
}

// Persistent: block w owns channel block (w % ncb) and every G-th spatial tile; BN statistics
// stay in registers until the segment changes (one flush per block and segment).
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void k_dw_fwd(DwArgs g) {
  constexpr int IH = (DTS - 1) * S + K, IW = IH;
  __shared__ __attribute__((aligned(16))) float tile[IH * IW * DCB];
  __shared__ __attribute__((aligned(16))) T otile[DTS * DTS * DCB];
  __shared__ float2 xf[DCB];
  __shared__ float gt[DCB];
  __shared__ float red[2][8][DCB];
  const int tid = threadIdx.x, c = tid & 31, r = tid >> 5;
  const int w = xcd_remap(blockIdx.x, gridDim.x);  // a pixel's channel blocks on one XCD
  const int cb = w % g.ncb, G = gridDim.x / g.ncb;
  const int c0 = cb * DCB;
  const bool cvalid = (c0 + c) < g.C;
  float wr[K * K];
  const T* Wp = (const T*)g.w;
  load_taps(wr, Wp, g.C, c0 + c, cvalid);
  T* Y = (T*)g.y;
  float s = 0.f, q = 0.f;
  int cur_seg = -1, xf_seg = -1, xf_img = -1;

  for (int t = w / g.ncb; t < g.tiles_total; t += G) {
    int seg, n, ty, tx;
    locate_tile(g.pout, t, seg, n, ty, tx);
    const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
    const int pt = same_pad(H, K, S), pl = same_pad(W, K, S);
    const int oy0 = ty * DTS, ox0 = tx * DTS;
    __syncthreads();  // previous tile's LDS readers are done
    if (seg != cur_seg) {
      if (cur_seg >= 0 && g.has_stats) {
        red[0][r][c] = s;
        red[1][r][c] = q;
        __syncthreads();
        if (tid < DCB && c0 + tid < g.C) {
          float ss = 0.f, qq = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) { ss += red[0][i][tid]; qq += red[1][i][tid]; }
          stat_put(g.stats.sum[cur_seg], c0 + tid, (double)(ss));
          stat_put(g.stats.sq[cur_seg], c0 + tid, (double)(qq));
        }
      }
      s = 0.f;
      q = 0.f;
      cur_seg = seg;
    }
    Stage<T, IH, IW> st;
    st.fetch(g, seg, n, oy0 * S - pt, ox0 * S - pl, c0);
    // affine / gate only when the segment / image changes (block-uniform): a block walks
    // ~20 tiles of one image, and the re-derivation was a dependent global round trip and a
    // barrier per tile
    if (seg != xf_seg || (g.lz.gate && n != xf_img)) {
      prep_xf(g, xf, gt, seg, n, c0);
      xf_seg = seg;
      xf_img = n;
      __syncthreads();
    }
    st.commit(g, tile, xf, gt);
    __syncthreads();

    float acc[DTS];
#pragma unroll
    for (int j = 0; j < DTS; ++j) acc[j] = 0.f;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const float wv = wr[kh * K + kw];
        const float* trow = tile + ((r * S + kh) * IW + kw) * DCB + c;
#pragma unroll
        for (int j = 0; j < DTS; ++j) acc[j] += trow[j * S * DCB] * wv;
      }
    const int oy = oy0 + r;
#pragma unroll
    for (int j = 0; j < DTS; ++j) {
      otile[(r * DTS + j) * DCB + c] = from_f<T>(acc[j]);
      if (oy < OH && ox0 + j < OW && cvalid) {
        s += acc[j];
        q += acc[j] * acc[j];
      }
    }
    __syncthreads();
    // one 16-byte vector per thread: pixel tid/4, channels (tid%4)*8 .. +8
    {
      const int px = tid >> 2, cv = (tid & 3) * 8;
      const int py = oy0 + (px >> 3), pxx = ox0 + (px & 7), nc = g.C - (c0 + cv);
      if (py < OH && pxx < OW && nc > 0) {
        const size_t o = ((size_t)g.pout.row_off[seg] + (size_t)n * OH * OW + (size_t)py * OW + pxx) * g.C + c0 + cv;
        if constexpr (sizeof(T) == 2) {
          if (nc >= 8) {
            *reinterpret_cast<uint4*>(Y + o) = *reinterpret_cast<const uint4*>(otile + px * DCB + cv);
          } else {
            for (int j = 0; j < nc; ++j) Y[o + j] = otile[px * DCB + cv + j];
          }
        } else {
          for (int j = 0; j < 8 && j < nc; ++j) Y[o + j] = otile[px * DCB + cv + j];
        }
      }
    }
  }
  if (cur_seg >= 0 && g.has_stats) {
    __syncthreads();
    red[0][r][c] = s;
    red[1][r][c] = q;
    __syncthreads();
    if (tid < DCB && c0 + tid < g.C) {
      float ss = 0.f, qq = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) { ss += red[0][i][tid]; qq += red[1][i][tid]; }
      stat_put(g.stats.sum[cur_seg], c0 + tid, (double)(ss));
      stat_put(g.stats.sq[cur_seg], c0 + tid, (double)(qq));
    }
  }
}

// dx[n][iy][ix][c] = sum_{kh,kw} dy[n][oy][ox][c] * w[kh][kw][c],  iy = oy*s - pt + kh
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void k_dw_dgrad(DwArgs g) {
  constexpr int HR = (DTS - 1 + K - 1) / S + 2;
  __shared__ __attribute__((aligned(16))) float tile[HR * HR * DCB];
  const int tid = threadIdx.x, c = tid & 31, r = tid >> 5;

  int id = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = id % g.ncb;
  id /= g.ncb;
  int seg, n, ty, tx;
  locate_tile(g.pin, id, seg, n, ty, tx);
  const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
  const int c0 = cb * DCB;
  const int pt = same_pad(H, K, S), pl = same_pad(W, K, S);
  const int iy0 = ty * DTS, ix0 = tx * DTS;
  const int oy_lo = fdiv(iy0 + pt - (K - 1) + S - 1, S);
  const int ox_lo = fdiv(ix0 + pl - (K - 1) + S - 1, S);

  const T* DY = (const T*)g.dy;
  const size_t obase = (size_t)g.pout.row_off[seg] + (size_t)n * OH * OW;
  for (int v = tid; v < HR * HR * (DCB / 8); v += 256) {
    const int pix = v >> 2, cv = (v & 3) * 8;
    const int yy = pix / HR, xx = pix - yy * HR;
    const int oy = oy_lo + yy, ox = ox_lo + xx, nc = g.C - (c0 + cv);
    float vals[8];
    if (oy >= 0 && oy < OH && ox >= 0 && ox < OW && nc > 0) ld8m(DY + (obase + (size_t)oy * OW + ox) * g.C + c0 + cv, nc, vals);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = 0.f;
    }
    float* d = tile + pix * DCB + cv;
    reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
    reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
  }
  float wr[K * K];
  const T* Wp = (const T*)g.w;
  const bool cvalid = (c0 + c) < g.C;
  load_taps(wr, Wp, g.C, c0 + c, cvalid);
  __syncthreads();

  const int iy = iy0 + r;
  float acc[DTS];
#pragma unroll
  for (int j = 0; j < DTS; ++j) acc[j] = 0.f;
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
    const int t = iy + pt - kh;
    if (t < 0 || (S > 1 && (t % S) != 0)) continue;
    const int ly = t / S - oy_lo;
#pragma unroll
    for (int kw = 0; kw < K; ++kw) {
      const float wv = wr[kh * K + kw];
#pragma unroll
      for (int j = 0; j < DTS; ++j) {
        const int u = ix0 + j + pl - kw;
        if (u < 0 || (S > 1 && (u % S) != 0)) continue;
        const int lx = u / S - ox_lo;
        acc[j] += tile[(ly * HR + lx) * DCB + c] * wv;
      }
    }
  }
  if (iy < H && cvalid) {
    T* DX = (T*)g.dx;
    const size_t ibase = (size_t)g.pin.row_off[seg] + (size_t)n * H * W;
#pragma unroll
    for (int j = 0; j < DTS; ++j) {
      const int ix = ix0 + j;
      if (ix < W) {
        T* p = DX + (ibase + (size_t)iy * W + ix) * g.C + c0 + c;
        *p = from_f<T>(g.accumulate ? to_f<T>(*p) + acc[j] : acc[j]);
      }
    }
  }
}

// dw[kh][kw][c] += sum_{n,oy,ox} dy[n][oy][ox][c] * v(x)[n][oy*s-pt+kh][ox*s-pl+kw][c]
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void k_dw_wgrad(DwArgs g) {
  constexpr int IH = (DTS - 1) * S + K, IW = IH;
  constexpr int TILE = IH * IW * DCB, RED = K * K * 8 * DCB;
  constexpr int LDSF = TILE > RED ? TILE : RED;
  __shared__ __attribute__((aligned(16))) float lds[LDSF];
  __shared__ float2 xf[DCB];
  __shared__ float gt[DCB];
  const int tid = threadIdx.x, c = tid & 31, r = tid >> 5;

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = bid % g.ncb;
  const int chunk = bid / g.ncb;
  const int c0 = cb * DCB;
  const bool cvalid = (c0 + c) < g.C;
  const int t_begin = chunk * g.tiles_per_wg;
  const int t_end = min(g.tiles_total, t_begin + g.tiles_per_wg);
  const T* DY = (const T*)g.dy;

  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  int xf_seg = -1, xf_img = -1;

  for (int t = t_begin; t < t_end; ++t) {
    int seg, n, ty, tx;
    locate_tile(g.pout, t, seg, n, ty, tx);
    const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
    const int pt = same_pad(H, K, S), pl = same_pad(W, K, S);
    const int oy0 = ty * DTS, ox0 = tx * DTS;
    __syncthreads();
    Stage<T, IH, IW> st;
    st.fetch(g, seg, n, oy0 * S - pt, ox0 * S - pl, c0);
    // this tile's dy values go out with the halo loads (select-predicated), not after commit
    const int oy = oy0 + r;
    const size_t obase = (size_t)g.pout.row_off[seg] + (size_t)n * OH * OW;
    // (a zero select on the loaded value let the compiler branch around each conversion with a
    // vmcnt(0) inside, draining the halo loads eight times per tile: zeroed by a multiply)
    T dyr[DTS];
    float dym[DTS];
#pragma unroll
    for (int j = 0; j < DTS; ++j) {
      const int ox = ox0 + j;
      const bool in = oy < OH && ox < OW && cvalid;
      dyr[j] = DY[in ? (obase + (size_t)oy * OW + ox) * g.C + c0 + c : 0];
      dym[j] = in ? 1.f : 0.f;
    }
    if (seg != xf_seg || (g.lz.gate && n != xf_img)) {  // block-uniform, as in k_dw_fwd
      prep_xf(g, xf, gt, seg, n, c0);
      xf_seg = seg;
      xf_img = n;
      __syncthreads();
    }
    st.commit(g, lds, xf, gt);
    float dyv[DTS];
#pragma unroll
    for (int j = 0; j < DTS; ++j) dyv[j] = to_f<T>(dyr[j]) * dym[j];
    __syncthreads();
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const float* trow = lds + ((r * S + kh) * IW + kw) * DCB + c;
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < DTS; ++j) a += dyv[j] * trow[j * S * DCB];
        acc[kh * K + kw] += a;
      }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < K * K; ++i) lds[(i * 8 + r) * DCB + c] = acc[i];
  __syncthreads();
  for (int e = tid; e < K * K * DCB; e += 256) {
    const int i = e / DCB, cc = e - i * DCB;
    if (c0 + cc < g.C) {
      float s = 0.f;
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) s += lds[(i * 8 + rr) * DCB + cc];
      if (g.part) g.part[((size_t)chunk * K * K + i) * g.C + c0 + cc] = s;
      else atomicAdd(g.dw + (size_t)i * g.C + c0 + cc, s);
    }
  }
}

// ------------------------------------------------------------------ pipelined tile forms
// Same work unit as k_dw_fwd / k_dw_wgrad (8x8 output tile x 32 channels, persistent over the
// tiles of one channel block), with the per-tile latency chain cut:
//   * the lazy BN affine is derived once per segment (it was re-derived from the fp64 sums for
//     every tile, a dependent global round trip before the tile's own loads could start);
//   * tile t+1's raw input vectors (and its SE gate values) are fetched into registers while
//     tile t is computed, then transformed into the other half of a double-buffered LDS tile;
//   * the stencil keeps one input row per kh in registers and reuses it for all K taps of that
//     row (K x (8*S+K-1) LDS reads per 8 outputs instead of K*K*8).
// wgrad stages dy through LDS the same way and needs one barrier per tile.
template <typename T, int K, int S, bool WGRAD>
__global__ __launch_bounds__(256) void k_dw3(DwArgs g) {
  constexpr int IH = (DTS - 1) * S + K, IW = IH, NPIX = IH * IW;
  constexpr int RW = (DTS - 1) * S + K;                 // input row window per output row
  constexpr int NV = (NPIX * (DCB / 8) + 255) / 256;    // staged vectors per thread
  constexpr int TILEF = NPIX * DCB;
  __shared__ __attribute__((aligned(16))) float tile[2][TILEF];
  __shared__ __attribute__((aligned(16))) float dyt[WGRAD ? 2 : 1][WGRAD ? DTS * DTS * DCB : 4];
  __shared__ __attribute__((aligned(16))) T otile[WGRAD ? 8 : DTS * DTS * DCB];
  __shared__ float2 xf[DCB];
  __shared__ float red[2][8][DCB];
  const int tid = threadIdx.x, c = tid & 31, r = tid >> 5;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = w % g.ncb, G = gridDim.x / g.ncb;
  const int c0 = cb * DCB;
  const int C = g.C;
  const bool cvalid = (c0 + c) < C;
  const int t0 = w / g.ncb;
  if (t0 >= g.tiles_total) return;
  const int nt = (g.tiles_total - 1 - t0) / G + 1;

  float wr[WGRAD ? 1 : K * K];
  if constexpr (!WGRAD) {
    const T* Wp = (const T*)g.w;
    load_taps(wr, Wp, C, c0 + c, cvalid);
  }
  const T* X = (const T*)g.x;
  const T* DY = (const T*)g.dy;
  const bool has_gate = g.lz.gate != nullptr;

  // ---- prefetch registers
  uint4 rx[NV][sizeof(T) == 2 ? 1 : 2];
  float4 rg[NV][2];
  uint4 rdy[sizeof(T) == 2 ? 1 : 2];
  int rvalid = 0;  // bit u: staged vector u is inside the image
  auto fetch = [&](int t) {
    int seg, n, ty, tx;
    locate_tile(g.pout, t, seg, n, ty, tx);
    const int H = g.pin.H[seg], W = g.pin.W[seg];
    const int iy0 = ty * DTS * S - same_pad(H, K, S), ix0 = tx * DTS * S - same_pad(W, K, S);
    const size_t base = (size_t)g.pin.row_off[seg] + (size_t)n * H * W;
    rvalid = 0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = tid + u * 256;
      const int pix = v >> 2, cv = (v & 3) * 8;
      const int yy = pix / IW, xx = pix - yy * IW;
      const int gy = iy0 + yy, gx = ix0 + xx;
      if (v < NPIX * 4 && gy >= 0 && gy < H && gx >= 0 && gx < W && c0 + cv < C) {
        const uint4* src = reinterpret_cast<const uint4*>(X + (base + (size_t)gy * W + gx) * g.lz.ld + c0 + cv);
        rx[u][0] = src[0];
        if constexpr (sizeof(T) == 4) rx[u][1] = src[1];
        if (has_gate) {
          const float4* gp = reinterpret_cast<const float4*>(g.lz.gate + (size_t)n * C + c0 + cv);
          rg[u][0] = gp[0];
          rg[u][1] = gp[1];
        }
        rvalid |= 1 << u;
      }
    }
    if constexpr (WGRAD) {  // dy tile: pixel tid/4 of the 8x8 tile, channels (tid%4)*8
      const int OH = g.pout.H[seg], OW = g.pout.W[seg];
      const int px = tid >> 2, cv = (tid & 3) * 8;
      const int oy = ty * DTS + (px >> 3), ox = tx * DTS + (px & 7);
      rdy[0] = make_uint4(0, 0, 0, 0);
      if constexpr (sizeof(T) == 4) rdy[1] = make_uint4(0, 0, 0, 0);
      if (oy < OH && ox < OW && c0 + cv < C) {
        const uint4* src = reinterpret_cast<const uint4*>(
            DY + ((size_t)g.pout.row_off[seg] + (size_t)n * OH * OW + (size_t)oy * OW + ox) * C + c0 + cv);
        rdy[0] = src[0];
        if constexpr (sizeof(T) == 4) rdy[1] = src[1];
      }
    }
  };
  auto unpack8 = [&](const uint4* q, float* o) {
    if constexpr (sizeof(T) == 2) {
      const uint32_t wv[4] = {q[0].x, q[0].y, q[0].z, q[0].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(wv[i] << 16);
        o[2 * i + 1] = __uint_as_float(wv[i] & 0xffff0000u);
      }
    } else {
      const uint32_t wv[8] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w};
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = __uint_as_float(wv[i]);
    }
  };
  auto commit = [&](int buf) {
    // this thread's 8 channels are the same for every u: affine in registers once
    const int cv0 = (tid & 3) * 8;
    float2 a8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a8[j] = xf[cv0 + j];
    const int act = g.lz.act;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = tid + u * 256;
      if (v >= NPIX * 4) break;
      const int pix = v >> 2, cv = (v & 3) * 8;
      float vals[8];
      if (rvalid & (1 << u)) {
        unpack8(rx[u], vals);
        const float gv[8] = {rg[u][0].x, rg[u][0].y, rg[u][0].z, rg[u][0].w, rg[u][1].x, rg[u][1].y, rg[u][1].z, rg[u][1].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          vals[j] = lazy_apply(vals[j], a8[j], act);
          if (has_gate) vals[j] *= gv[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[j] = 0.f;
      }
      float* d = &tile[buf][pix * DCB + cv];
      reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
      reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
    }
    if constexpr (WGRAD) {
      float vals[8];
      unpack8(rdy, vals);
      float* d = &dyt[buf][tid * 8];  // [pixel][32] with pixel = tid/4, channels (tid%4)*8
      reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
      reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
    }
  };
  int xf_seg = -1;
  auto ensure_affine = [&](int seg) {  // block-uniform; rare (segment changes)
    if (seg == xf_seg) return;
    __syncthreads();
    if (tid < DCB) {
      const int cc = c0 + tid;
      xf[tid] = cc < C ? bn_affine(g.lz.bn, seg, cc, 1.f / (float)seg_rows(g.pin, seg)) : make_float2(1.f, 0.f);
    }
    __syncthreads();
    xf_seg = seg;
  };
  auto tile_seg = [&](int t) {
    int seg, n, ty, tx;
    locate_tile(g.pout, t, seg, n, ty, tx);
    return seg;
  };

  float s = 0.f, q = 0.f;  // fwd BN statistics of channel c
  float acc[WGRAD ? K * K : 1];
#pragma unroll
  for (int i = 0; i < (WGRAD ? K * K : 1); ++i) acc[i] = 0.f;
  int cur_seg = -1;
  auto flush_stats = [&](int seg) {  // block-uniform
    __syncthreads();
    red[0][r][c] = s;
    red[1][r][c] = q;
    __syncthreads();
    if (tid < DCB && c0 + tid < C) {
      float ss = 0.f, qq = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) { ss += red[0][i][tid]; qq += red[1][i][tid]; }
      stat_put(g.stats.sum[seg], c0 + tid, (double)ss);
      stat_put(g.stats.sq[seg], c0 + tid, (double)qq);
    }
    s = 0.f;
    q = 0.f;
  };

  fetch(t0);
  ensure_affine(tile_seg(t0));
  commit(0);
  __syncthreads();
  for (int i = 0; i < nt; ++i) {
    const int t = t0 + i * G, buf = i & 1;
    const bool more = i + 1 < nt;
    int seg, n, ty, tx;
    locate_tile(g.pout, t, seg, n, ty, tx);
    if (!WGRAD && g.has_stats && seg != cur_seg) {
      if (cur_seg >= 0) flush_stats(cur_seg);
      cur_seg = seg;
    }
    if (more) fetch(t + G);
    const float* tb = tile[buf];
    if constexpr (!WGRAD) {
      float o[DTS];
#pragma unroll
      for (int j = 0; j < DTS; ++j) o[j] = 0.f;
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        float rowv[RW];
        const float* trow = tb + ((r * S + kh) * IW) * DCB + c;
#pragma unroll
        for (int x = 0; x < RW; ++x) rowv[x] = trow[x * DCB];
#pragma unroll
        for (int kw = 0; kw < K; ++kw)
#pragma unroll
          for (int j = 0; j < DTS; ++j) o[j] += rowv[j * S + kw] * wr[kh * K + kw];
      }
      const int OH = g.pout.H[seg], OW = g.pout.W[seg];
      const int oy = ty * DTS + r;
#pragma unroll
      for (int j = 0; j < DTS; ++j) {
        otile[(r * DTS + j) * DCB + c] = from_f<T>(o[j]);
        if (oy < OH && tx * DTS + j < OW && cvalid) { s += o[j]; q += o[j] * o[j]; }
      }
      __syncthreads();
      {
        const int px = tid >> 2, cv = (tid & 3) * 8;
        const int py = ty * DTS + (px >> 3), pxx = tx * DTS + (px & 7);
        if (py < OH && pxx < OW && c0 + cv < C) {
          T* Y = (T*)g.y;
          const size_t o_ = ((size_t)g.pout.row_off[seg] + (size_t)n * OH * OW + (size_t)py * OW + pxx) * C + c0 + cv;
          if constexpr (sizeof(T) == 2) {
            *reinterpret_cast<uint4*>(Y + o_) = *reinterpret_cast<const uint4*>(otile + px * DCB + cv);
          } else {
            *reinterpret_cast<float4*>(Y + o_) = *reinterpret_cast<const float4*>(otile + px * DCB + cv);
            *reinterpret_cast<float4*>(Y + o_ + 4) = *reinterpret_cast<const float4*>(otile + px * DCB + cv + 4);
          }
        }
      }
    } else {
      float dyv[DTS];
#pragma unroll
      for (int j = 0; j < DTS; ++j) dyv[j] = cvalid ? dyt[buf][(r * DTS + j) * DCB + c] : 0.f;
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        float rowv[RW];
        const float* trow = tb + ((r * S + kh) * IW) * DCB + c;
#pragma unroll
        for (int x = 0; x < RW; ++x) rowv[x] = trow[x * DCB];
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          float a = 0.f;
#pragma unroll
          for (int j = 0; j < DTS; ++j) a += dyv[j] * rowv[j * S + kw];
          acc[kh * K + kw] += a;
        }
      }
    }
    if (more) {
      ensure_affine(tile_seg(t + G));
      commit(buf ^ 1);
    }
    __syncthreads();
  }
  if constexpr (!WGRAD) {
    if (g.has_stats && cur_seg >= 0) flush_stats(cur_seg);
  } else {
    // block reduction of the K*K x 32 filter partials over the 8 row-threads (both tile
    // buffers are free now and contiguous)
    static_assert(K * K * 8 <= 2 * NPIX, "wgrad reduction scratch exceeds the tile buffers");
    float* lds = &tile[0][0];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < K * K; ++i) lds[(i * 8 + r) * DCB + c] = acc[i];
    __syncthreads();
    for (int e = tid; e < K * K * DCB; e += 256) {
      const int i = e / DCB, cc = e - i * DCB;
      if (c0 + cc < C) {
        float sum = 0.f;
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) sum += lds[(i * 8 + rr) * DCB + cc];
        atomicAdd(g.dw + (size_t)i * C + c0 + cc, sum);
      }
    }
  }
}

// ------------------------------------------------------------------ direct (barrier-free) forms
// One thread = one output pixel x one 8-channel vector; the K*K taps are 16-byte loads served
// by L1/L2 (each input vector is reused by the neighbouring pixels' threads), transformed,
// multiplied and accumulated in registers; one 16-byte store.  A block is R pixel rows of
// TPR = C/8 threads, so every thread keeps one channel vector for the whole launch: the lazy
// affine lives in registers and the BN statistics are per-thread partials, reduced once per
// segment.  No LDS staging, no barriers inside the pixel loop.
struct DwGeom {
  int TPR, R;  // threads per pixel (C/8), pixels per block pass
  int ncs;     // k_dw4_dgrad: channel splits per pixel (consecutive blocks)
};
static DwGeom dw_geom(int C) {
  DwGeom d;
  d.TPR = C / 8;
  d.R = std::max(1, 256 / d.TPR);
  d.ncs = 1;
  return d;
}

template <typename T, int K, int S>
__global__ __launch_bounds__(256) void k_dw2_fwd(DwArgs g, DwGeom geo) {
  extern __shared__ float red2[];  // [2][R][C] statistics partials
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  const bool act_thread = rr < geo.R;
  const int c = tv * 8, C = g.C;
  const T* X = (const T*)g.x;
  const T* Wt = (const T*)g.w;
  T* Y = (T*)g.y;
  for (int seg = 0; seg < g.pout.nseg; ++seg) {
    const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
    const int pt = same_pad(H, K, S), pl = same_pad(W, K, S);
    const int npix = g.pout.batch * OH * OW;
    float2 af[8];
    const float inv = 1.f / (float)seg_rows(g.pin, seg);
#pragma unroll
    for (int j = 0; j < 8; ++j) af[j] = bn_affine(g.lz.bn, seg, c + j, inv);
    float s[8], q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
    if (act_thread) {
      for (int p = blockIdx.x * geo.R + rr; p < npix; p += gridDim.x * geo.R) {
        const int n = p / (OH * OW), rem = p - n * (OH * OW);
        const int oy = rem / OW, ox = rem - oy * OW;
        const size_t ibase = (size_t)g.pin.row_off[seg] + (size_t)n * H * W;
        float gt[8];
        if (g.lz.gate) ld8(g.lz.gate + (size_t)n * C + c, gt);
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
        for (int kh = 0; kh < K; ++kh) {
          const int iy = oy * S - pt + kh;
          if (iy < 0 || iy >= H) continue;
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            const int ix = ox * S - pl + kw;
            if (ix < 0 || ix >= W) continue;
            float xv[8], wv[8];
            ld8(X + (ibase + (size_t)iy * W + ix) * g.lz.ld + c, xv);
            ld8(Wt + (size_t)(kh * K + kw) * C + c, wv);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float v = lazy_apply(xv[j], af[j], g.lz.act);
              if (g.lz.gate) v *= gt[j];
              acc[j] += v * wv[j];
            }
          }
        }
        st8(Y + ((size_t)g.pout.row_off[seg] + p) * C + c, acc);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] += acc[j]; q[j] += acc[j] * acc[j]; }
      }
    }
    if (g.has_stats) {  // fixed-order block reduction, one fp64 atomic per channel
      if (act_thread)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          red2[rr * C + c + j] = s[j];
          red2[(geo.R + rr) * C + c + j] = q[j];
        }
      __syncthreads();
      for (int ch = tid; ch < C; ch += blockDim.x) {
        float ss = 0.f, qq = 0.f;
        for (int i = 0; i < geo.R; ++i) { ss += red2[i * C + ch]; qq += red2[(geo.R + i) * C + ch]; }
        stat_put(g.stats.sum[seg], ch, (double)ss);
        stat_put(g.stats.sq[seg], ch, (double)qq);
      }
      __syncthreads();
    }
  }
}

// dx[n][iy][ix][c] (+)= sum over taps (kh, kw) with iy = oy*S - pt + kh of dy[n][oy][ox][c] * w
template <typename T, int K, int S>
__global__ __launch_bounds__(256) void k_dw2_dgrad(DwArgs g, DwGeom geo) {
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  if (rr >= geo.R) return;
  const int c = tv * 8, C = g.C;
  const T* DY = (const T*)g.dy;
  const T* Wt = (const T*)g.w;
  T* DX = (T*)g.dx;
  for (int seg = 0; seg < g.pin.nseg; ++seg) {
    const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
    const int pt = same_pad(H, K, S), pl = same_pad(W, K, S);
    const int npix = g.pin.batch * H * W;
    for (int p = blockIdx.x * geo.R + rr; p < npix; p += gridDim.x * geo.R) {
      const int n = p / (H * W), rem = p - n * (H * W);
      const int iy = rem / W, ix = rem - iy * W;
      const size_t obase = (size_t)g.pout.row_off[seg] + (size_t)n * OH * OW;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
      for (int kh = 0; kh < K; ++kh) {
        const int ty = iy + pt - kh;
        if (ty < 0 || (S > 1 && (ty % S) != 0)) continue;
        const int oy = ty / S;
        if (oy >= OH) continue;
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          const int tx = ix + pl - kw;
          if (tx < 0 || (S > 1 && (tx % S) != 0)) continue;
          const int ox = tx / S;
          if (ox >= OW) continue;
          float dv[8], wv[8];
          ld8(DY + (obase + (size_t)oy * OW + ox) * C + c, dv);
          ld8(Wt + (size_t)(kh * K + kw) * C + c, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += dv[j] * wv[j];
        }
      }
      acc8m(DX + ((size_t)g.pin.row_off[seg] + p) * C + c, 8, acc, g.accumulate);
    }
  }
}

// ------------------------------------------------------------------ register-blocked dgrad
// One thread = one PH x PW patch of dx pixels x CPT channels; the K*K weights of its channels
// live in registers as fp32 for the whole launch.  Patches start on u = iy + pt multiples of S,
// so which dy pixel pairs with which (dx pixel, tap) is known at compile time:
//   dy row = A + (e - kh) / S  for (e - kh) % S == 0   (A = patch row / S, e = row in patch)
// Every dy vector the patch needs is loaded and unpacked once and feeds all its taps (k3 s2:
// 4 loads for 4 dx pixels, against 9 tap loads + 9 weight loads per pixel in k_dw2_dgrad).
template <int CPT, typename T> __device__ __forceinline__ void ldv(const T* p, float* o) {
  if constexpr (CPT == 8) {
    ld8(p, o);
  } else if constexpr (CPT == 2) {
    if constexpr (sizeof(T) == 2) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(p);
      o[0] = __uint_as_float(v << 16); o[1] = __uint_as_float(v & 0xffff0000u);
    } else {
      const float2 a = *reinterpret_cast<const float2*>(p);
      o[0] = a.x; o[1] = a.y;
    }
  } else if constexpr (sizeof(T) == 2) {
    uint2 v = *reinterpret_cast<const uint2*>(p);
    o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
    o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  } else {
    float4 a = *reinterpret_cast<const float4*>(p);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  }
}
template <int CPT, typename T> __device__ __forceinline__ void stv(T* p, const float* v) {
  if constexpr (CPT == 8) {
    st8(p, v);
  } else if constexpr (CPT == 2) {
    if constexpr (sizeof(T) == 2) *reinterpret_cast<uint32_t*>(p) = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    else *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                              (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// FOLD (accumulate == 0): dx is the gradient of the lazy value g.lz = act(bn(x)); the thread also
// takes that BatchNorm's backward sums of its channels (du = dx * act'(bn(x)) from the stored dx,
// dbeta += du, dgamma += du * xhat), reduced over the block's pixel rows in a fixed order at the end
// of every segment and flushed as one fp64 atomic per channel -- the edet_lazy_bwd_reduce pass over
// (x, dx) folded into the launch that writes dx (mb_conv_block.py:143-147 backward at stride 2)
template <typename T, int K, int S, int CPT, int PH, int PW, bool FOLD = false>
__global__ __launch_bounds__(256) void k_dw4_dgrad(DwArgs g, DwGeom geo, edet_bngrad64 fold) {
  static_assert(PH % S == 0 && PW % S == 0, "patch must cover whole strides");
  constexpr int DLO = -((K - 1) / S), DHR = (PH - 1) / S, DHC = (PW - 1) / S;
  extern __shared__ float fred[];  // FOLD: [TPR * CPT] float4 tables, then [2][R][TPR * CPT] sums
  float4* ftab = reinterpret_cast<float4*>(fred);
  float* fsum = fred + 4 * geo.TPR * CPT;
  const int tid = threadIdx.x, rr = tid / geo.TPR, tv = tid - rr * geo.TPR;
  if (rr >= geo.R) return;  // (never: the block is TPR x R threads)
  // channel splits innermost (geo.ncs consecutive logical blocks = one XCD, the same pixels)
  const int bx = xcd_remap(blockIdx.x, gridDim.x), cs = bx % geo.ncs, pb = bx / geo.ncs;
  const int pgrid = gridDim.x / geo.ncs;
  const int c = (cs * geo.TPR + tv) * CPT, C = g.C;
  const T* DY = (const T*)g.dy;
  T* DX = (T*)g.dx;
  const T* X = (const T*)g.lz.x;
  float w[K * K][CPT];
#pragma unroll
  for (int i = 0; i < K * K; ++i) ldv<CPT>((const T*)g.w + (size_t)i * C + c, w[i]);
  for (int seg = 0; seg < g.pin.nseg; ++seg) {
    const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
    const int pt = same_pad(H, K, S), pl = same_pad(W, K, S);
    const int PR = cdiv(H + pt, PH), PC = cdiv(W + pl, PW), per_img = PR * PC;
    const int npatch = g.pin.batch * per_img;
    // FOLD: per channel (scale, shift, mean, rstd) in LDS (registers would cost the occupancy
    // the patch loop needs), partial sums in registers
    float fs[CPT], fq[CPT];
    if constexpr (FOLD) {
      const float inv = 1.f / (float)seg_rows(g.pin, seg);
      for (int e = tid; e < geo.TPR * CPT; e += blockDim.x) {
        const int ch = cs * geo.TPR * CPT + e;
        const float2 af = bn_affine(g.lz.bn, seg, ch, inv), mr = bn_mean_rstd(g.lz.bn, seg, ch, inv);
        ftab[e] = make_float4(af.x, af.y, mr.x, mr.y);
      }
#pragma unroll
      for (int j = 0; j < CPT; ++j) { fs[j] = 0.f; fq[j] = 0.f; }
      __syncthreads();
    }
    // FOLD: a patch's x vectors are requested one patch ahead (raw, select-predicated): their
    // latency hides behind the current patch's dy loads and taps
    using XR = typename std::conditional<sizeof(T) == 2, uint32_t, float>::type;
    constexpr int XW = sizeof(T) == 2 ? CPT / 2 : CPT;  // raw words per CPT channels
    XR xnext[FOLD ? PH : 1][FOLD ? PW : 1][XW];
    auto fetch_x = [&](int qq) {
      if constexpr (FOLD) {
        const bool live = qq < npatch;
        const int n = live ? qq / per_img : 0, rem = live ? qq - n * per_img : 0;
        const int pr = rem / PC, pc = rem - pr * PC;
        const T* xb = X + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * g.lz.ld + c;
#pragma unroll
        for (int e = 0; e < PH; ++e)
#pragma unroll
          for (int f = 0; f < PW; ++f) {
            const int iy = pr * PH + e - pt, ix = pc * PW + f - pl;
            const bool ok = live && iy >= 0 && iy < H && ix >= 0 && ix < W;
            const XR* p = reinterpret_cast<const XR*>(xb + (ok ? (uint32_t)((iy * W + ix) * g.lz.ld) : 0u));
#pragma unroll
            for (int w = 0; w < XW; ++w) xnext[e][f][w] = p[w];
          }
      }
    };
    fetch_x(pb * geo.R + rr);
    for (int q = pb * geo.R + rr; q < npatch; q += pgrid * geo.R) {
      const int n = q / per_img, rem = q - n * per_img;
      const int pr = rem / PC, pc = rem - pr * PC;
      const int A = pr * (PH / S), Bc = pc * (PW / S);
      float xv[FOLD ? PH : 1][FOLD ? PW : 1][CPT];
      if constexpr (FOLD) {
#pragma unroll
        for (int e = 0; e < PH; ++e)
#pragma unroll
          for (int f = 0; f < PW; ++f)
#pragma unroll
            for (int w = 0; w < XW; ++w) {
              if constexpr (sizeof(T) == 2) {
                xv[e][f][2 * w] = __uint_as_float(xnext[e][f][w] << 16);
                xv[e][f][2 * w + 1] = __uint_as_float(xnext[e][f][w] & 0xffff0000u);
              } else {
                xv[e][f][w] = xnext[e][f][w];
              }
            }
        fetch_x(q + pgrid * geo.R);
      }
      const T* dyb = DY + ((size_t)g.pout.row_off[seg] + (size_t)n * OH * OW) * C + c;
      float acc[PH][PW][CPT];
#pragma unroll
      for (int e = 0; e < PH; ++e)
#pragma unroll
        for (int f = 0; f < PW; ++f)
#pragma unroll
          for (int j = 0; j < CPT; ++j) acc[e][f][j] = 0.f;
      // loads are predicated by select, not branched around: a load inside a divergent `if`
      // is waited on before the join, which serialises the K*K-ish loads of a k5 patch
#pragma unroll
      for (int dr = DLO; dr <= DHR; ++dr) {
        const int oy = A + dr;
        const bool rok = oy >= 0 && oy < OH;
#pragma unroll
        for (int dc = DLO; dc <= DHC; ++dc) {
          const int ox = Bc + dc;
          const bool ok = rok && ox >= 0 && ox < OW;
          float v[CPT];
          ldv<CPT>(dyb + (ok ? (uint32_t)((oy * OW + ox) * C) : 0u), v);
#pragma unroll
          for (int j = 0; j < CPT; ++j) v[j] = ok ? v[j] : 0.f;
#pragma unroll
          for (int e = 0; e < PH; ++e) {
            const int kh = e - S * dr;
            if (kh < 0 || kh >= K) continue;
#pragma unroll
            for (int f = 0; f < PW; ++f) {
              const int kw = f - S * dc;
              if (kw < 0 || kw >= K) continue;
#pragma unroll
              for (int j = 0; j < CPT; ++j) acc[e][f][j] += v[j] * w[kh * K + kw][j];
            }
          }
        }
      }
      T* dxb = DX + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * C + c;
#pragma unroll
      for (int e = 0; e < PH; ++e) {
        const int iy = pr * PH + e - pt;
        if (iy < 0 || iy >= H) continue;
#pragma unroll
        for (int f = 0; f < PW; ++f) {
          const int ix = pc * PW + f - pl;
          if (ix < 0 || ix >= W) continue;
          T* p = dxb + (uint32_t)((iy * W + ix) * C);
          if (g.accumulate) {
            float o[CPT];
            ldv<CPT>(p, o);
#pragma unroll
            for (int j = 0; j < CPT; ++j) acc[e][f][j] += o[j];
          }
          stv<CPT>(p, acc[e][f]);
          if constexpr (FOLD) {
#pragma unroll
            for (int j = 0; j < CPT; ++j) {
              const float4 t = ftab[tv * CPT + j];
              const float y = to_f<T>(from_f<T>(acc[e][f][j])), x = xv[e][f][j];
              const float du = g.lz.act ? y * dswishf_(x * t.x + t.y) : y;
              fs[j] += du;
              fq[j] += du * ((x - t.z) * t.w);
            }
          }
        }
      }
    }
    if constexpr (FOLD) {  // fixed-order block reduction, one fp64 atomic per channel and sum
      const int CB = geo.TPR * CPT, cl = tv * CPT;
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        fsum[rr * CB + cl + j] = fs[j];
        fsum[(geo.R + rr) * CB + cl + j] = fq[j];
      }
      __syncthreads();
      for (int ch = tid; ch < CB; ch += blockDim.x) {
        float a = 0.f, b = 0.f;
        for (int i = 0; i < geo.R; ++i) { a += fsum[i * CB + ch]; b += fsum[(geo.R + i) * CB + ch]; }
        stat_put(fold.dbeta[seg], cs * CB + ch, (double)a);
        stat_put(fold.dgamma[seg], cs * CB + ch, (double)b);
      }
      __syncthreads();
    }
  }
}

template <typename T, int K, int S, bool FOLD = false>
static int launch_dw4_dgrad(const DwArgs& g, hipStream_t s, const edet_bngrad64* fold = nullptr) {
  // k5: 4 channels per thread (25 fp32 weights each in registers); 2 channels measured
  // faster only at C = 1152.  The fold's x vectors and sums need registers: 4 channels at k3 too
  constexpr int CPT = FOLD ? 4 : (K == 3 ? 8 : 4);
  DwGeom geo;
  // channel vectors per pixel row split over blockIdx.y until a row fits a block
  int ncs = 1;
  while (g.C / CPT / ncs > 256 || (g.C / CPT) % ncs) ++ncs;
  geo.TPR = g.C / CPT / ncs;
  geo.R = std::max(1, 256 / geo.TPR);
  geo.ncs = ncs;
  long patches = 0;
  for (int i = 0; i < g.pin.nseg; ++i) {
    const int pt = same_pad(g.pin.H[i], K, S), pl = same_pad(g.pin.W[i], K, S);
    patches += (long)g.pin.batch * cdiv(g.pin.H[i] + pt, 2) * cdiv(g.pin.W[i] + pl, 2);
  }
  // block cap (kbench sweep, round 2): 4096 for k3; the k5 patches carry 4x the work, fewer
  // blocks won there (8192 x 1152: 46.8 -> 40.5 us at 1024, 32768 x 480: 51.5 -> 43.2 at 2048)
  int cap = 4096;
  long rows_in = 0;
  for (int i = 0; i < g.pin.nseg; ++i) rows_in += (long)g.pin.batch * g.pin.H[i] * g.pin.W[i];
  if (K == 5) cap = rows_in <= 8192 ? 1024 : 2048;
  // round 3 (profiles/r03af_launch_size_sweep.txt): 1024 up to 32768 input rows at k5 (8192 x 672
  // out: 29.9 -> 24.1 us) and up to 131072 at k3 (32768 x 240 out: 21.1 -> 17.8 us)
  if ((K == 5 && rows_in <= 32768) || (K == 3 && rows_in <= 131072)) cap = 1024;
  if (dev_knob(14) > 0) cap = dev_knob(14);
  const int grid = (int)std::max<long>(1, std::min<long>(cap, (patches + geo.R - 1) / geo.R));
  const edet_bngrad64 fd = fold ? *fold : edet_bngrad64{};
  const size_t lds = FOLD ? (4 + 2 * (size_t)geo.R) * geo.TPR * CPT * sizeof(float) : 0;
  if (patches)
    EDET_LAUNCH((k_dw4_dgrad<T, K, S, CPT, 2, 2, FOLD>), dim3(grid * ncs), dim3(geo.TPR * geo.R), lds, s, g, geo, fd);
  return check_launch("edet dwconv dgrad");
}

template <typename T, int K, int S, bool WG>
static int launch_dw3(DwArgs g, hipStream_t s) {
  constexpr int IH = (DTS - 1) * S + K, NPIX = IH * IH;
  constexpr size_t lds = 2 * NPIX * DCB * 4 + (WG ? 2 * DTS * DTS * DCB * 4 : DTS * DTS * DCB * sizeof(T)) + 2 * 8 * DCB * 4 + 256;
  const int per_cu = (int)std::max<size_t>(1, std::min<size_t>(8, (160 * 1024) / lds));
  g.tiles_total = host_tiles(g.pout);
  if (!g.tiles_total) return EDET_OK;
  const int G = std::max(1, std::min(g.tiles_total, cdiv(256 * per_cu, g.ncb)));
  EDET_LAUNCH((k_dw3<T, K, S, WG>), dim3(G * g.ncb), dim3(256), 0, s, g);
  return check_launch("edet dwconv3");
}

// ------------------------------------------------------------------ row-streaming forms
// One workgroup = one image x 32 channels x a strip of TW = 8*CPG output columns x up to TH
// output rows.  It walks down its rows keeping the last K+S transformed input rows of the
// strip in an LDS ring, so every input element of the strip is loaded and transformed once
// (halo: (TW-1)*S+K columns per TW*S, K-S rows per block) against 2.25x in the 8x8 tiles for
// k5.  The S input rows of step i+1 (and, for wgrad, its dy row) are fetched into registers
// during step i-1 and committed to LDS during step i; one barrier per output row.
//   forward: each output row leaves through a double-buffered LDS stage as 16-byte stores;
//            BN statistics stay in registers until the block ends.
//   wgrad:   thread (c, column group) accumulates its K*K taps over the block's rows; the
//            column groups are reduced in LDS and added to dw once per block.
// The block count the rows per block are chosen for: scripts/dw_sweep.py over the D0 b32
// shapes, 1024 was best or within 3 % of best everywhere (3072 lost 10-20 %); prefetching 2-4
// steps ahead instead of 1 gained nothing.
constexpr int DWS_BLOCKS = 1024;
struct DwsPlan {
  int TH;                      // output rows per block
  int strips[EDET_MAX_SEG];    // column strips per segment
  int rowblk[EDET_MAX_SEG];    // row blocks per segment
  int nblk[EDET_MAX_SEG];      // blocks per segment (ncb * batch * rowblk * strips)
  int cb_inner;                // channel block innermost in the block order (see k_dws)
};

template <int N, int WORDS>
struct DwRaw {  // raw input vectors of a fetch, in registers until their commit
  static constexpr int NV = N;
  uint4 v[N][WORDS];
  uint32_t ok;
};

template <typename T, int K, int S, int CPG, bool WG, int P, int PF = 1, bool RB = false, bool SQ = false>
__global__ __launch_bounds__(256) void k_dws(DwArgs g, DwsPlan pl) {
  static_assert(PF == 1 || (PF == 2 && !WG), "two steps in flight: forward only");
  // SQ (inference): the SE squeeze of the output's value v(y) = act(bn(y)) in the epilogue --
  // with moving statistics bn's affine is known before the launch (layers/se.py:36 on
  // mb_conv_block.py:147-150 in call(training=False)), so the edet_se_squeeze pass is not needed
  static_assert(!SQ || !WG, "squeeze: forward only");
  // RB: the ring holds the transformed input rounded to bf16 (as the GEMMs stage their lazy A
  // operand) -- half the LDS, so more blocks per CU; forward with bf16 storage only
  static_assert(!RB || (!WG && sizeof(T) == 2), "bf16 ring: bf16 forward only");
  using RT = typename std::conditional<RB, uint16_t, float>::type;
  // P output rows per step: they share (P-1)*S... of their K input rows, so each input row of
  // the step is read from LDS once for all of them, and one barrier serves P rows
  constexpr int TW = 8 * CPG, IWS = (TW - 1) * S + K;
  constexpr int NR = (P - 1) * S + K;             // input rows one step reads
  constexpr int R = NR + P * S;                   // ring: those + the next step's new rows
  constexpr int RV = IWS * (DCB / 8);             // 8-channel vectors per input row
  constexpr int NVS = (P * S * RV + 255) / 256;   // per thread, P*S rows (one step)
  constexpr int NVP = (NR * RV + 255) / 256;      // per thread, NR rows (block prologue)
  constexpr int WORDS = sizeof(T) == 2 ? 1 : 2;
  constexpr int WIN = (CPG - 1) * S + K;
  static_assert(R * IWS >= 8 * K, "wgrad reduction scratch exceeds the ring");
  static_assert(R * IWS * DCB * sizeof(RT) >= 24 * DCB * sizeof(float), "statistics scratch exceeds the ring");
  __shared__ __attribute__((aligned(16))) RT ringb[R * IWS * DCB];
  float* ring = reinterpret_cast<float*>(ringb);  // the fp32 view (RB: end-of-block scratch only)
  __shared__ __attribute__((aligned(16))) T ost[WG ? 1 : 2][WG ? 8 : P * TW * DCB];  // fwd output stage
  __shared__ __attribute__((aligned(16))) float dys[WG ? 2 : 1][WG ? P * TW * DCB : 4];  // wgrad dy rows
  __shared__ float2 xf[DCB];
  __shared__ float gt[DCB];
  const int tid = threadIdx.x, c = tid & 31, gc = tid >> 5;

  // ---- block -> (seg, cb, n, row block, strip); consecutive logical ids share an XCD.
  // A block reads 32 channels = 64 B of each pixel, half of a 128-B line when C >= 64; with
  // the channel block innermost the blocks reading the other parts of the same lines are
  // consecutive logical ids, i.e. the same XCD (L2) at about the same time.
  int id = xcd_remap(blockIdx.x, gridDim.x), seg = 0;
  while (seg < g.pout.nseg - 1 && id >= pl.nblk[seg]) id -= pl.nblk[seg++];
  int cb = 0;
  if (pl.cb_inner) {
    cb = id % g.ncb;
    id /= g.ncb;
  }
  const int strip = id % pl.strips[seg];
  id /= pl.strips[seg];
  const int rb = id % pl.rowblk[seg];
  id /= pl.rowblk[seg];
  const int n = id % g.pout.batch;
  if (!pl.cb_inner) cb = id / g.pout.batch;
  const int c0 = cb * DCB, C = g.C;
  const int OH = g.pout.H[seg], OW = g.pout.W[seg], H = g.pin.H[seg], W = g.pin.W[seg];
  const int oy0 = rb * pl.TH, ox0 = strip * TW;
  const int nrows = min(pl.TH, OH - oy0);
  const int nsteps = cdiv(nrows, P);
  const int iy0 = oy0 * S - same_pad(H, K, S), ix0 = ox0 * S - same_pad(W, K, S);
  const size_t obase = (size_t)g.pout.row_off[seg] + (size_t)n * OH * OW;
  const T* X = (const T*)g.x + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * g.lz.ld + c0;
  const bool cvalid = c0 + c < C;

  float wr[WG ? 1 : K * K];
  if constexpr (!WG) load_taps(wr, (const T*)g.w, C, c0 + c, cvalid);
  if (tid < DCB) {
    const int cc = c0 + tid;
    xf[tid] = cc < C ? bn_affine(g.lz.bn, seg, cc, 1.f / (float)seg_rows(g.pin, seg)) : make_float2(1.f, 0.f);
    gt[tid] = (g.lz.gate && cc < C) ? g.lz.gate[(size_t)n * C + cc] : 1.f;
  }
  float2 ya = make_float2(1.f, 0.f);  // SQ: the output's affine for this thread's channel
  if constexpr (SQ) {
    if (cvalid) ya = bn_affine(g.yv.bn, seg, c0 + c, 1.f / (float)seg_rows(g.pout, seg));
  }
  float z = 0.f;  // SQ: sum of v(y) over the block's outputs of channel c

  // input rows [r0, r0 + nr) of the block (relative to iy0) <-> registers <-> ring slots
  auto fetch = [&](auto& rg, int r0, int nr) {
    constexpr int NV = std::remove_reference_t<decltype(rg)>::NV;
    rg.ok = 0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = tid + u * 256;
      const int row = v / RV, rem = v - row * RV, x = rem >> 2, cv = (rem & 3) * 8;
      const int gy = iy0 + r0 + row, gx = ix0 + x;
      const bool in = row < nr && gy >= 0 && gy < H && gx >= 0 && gx < W && c0 + cv < C;
      const uint4* src = reinterpret_cast<const uint4*>(X + (in ? (size_t)(gy * W + gx) * g.lz.ld + cv : 0));
      rg.v[u][0] = src[0];
      if constexpr (WORDS == 2) rg.v[u][1] = src[1];
      rg.ok |= (uint32_t)in << u;
    }
  };
  auto unpack8 = [&](const uint4* q, float* o) {
    if constexpr (WORDS == 1) {
      const uint32_t w4[4] = {q[0].x, q[0].y, q[0].z, q[0].w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[2 * i] = __uint_as_float(w4[i] << 16);
        o[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
      }
    } else {
      const uint32_t w8[8] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w};
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = __uint_as_float(w8[i]);
    }
  };
  auto commit = [&](const auto& rg, int r0, int nr) {
    constexpr int NV = std::remove_reference_t<decltype(rg)>::NV;
    const int cv0 = (tid & 3) * 8;  // the same 8 channels for every u (256 % 4 == 0)
    float2 a8[8];
    float g8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a8[j] = xf[cv0 + j]; g8[j] = gt[cv0 + j]; }
    const int act = g.lz.act;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = tid + u * 256;
      const int row = v / RV, rem = v - row * RV, x = rem >> 2;
      if (row >= nr) break;
      float vals[8];
      unpack8(rg.v[u], vals);
      // transform unconditionally and zero the padding by a multiply: a select lets the
      // compiler branch around the transform per element, and its vmcnt(0) inside those
      // branches drains the prefetch in flight (the raw vector of a padding slot is a real,
      // finite input element, see fetch)
      const float m = ((rg.ok >> u) & 1) ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = lazy_apply(vals[j], a8[j], act) * (g8[j] * m);
      int slot = (r0 % R) + row;
      if (slot >= R) slot -= R;
      RT* d = ringb + (slot * IWS + x) * DCB + cv0;
      if constexpr (RB) {
        uint32_t w4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) w4[i] = (uint32_t)f2bf(vals[2 * i]) | ((uint32_t)f2bf(vals[2 * i + 1]) << 16);
        *reinterpret_cast<uint4*>(d) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      } else {
        reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
        reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
      }
    }
  };
  // wgrad: the P dy rows of step j; vector e = tid + u*256: row e / (4 TW), pixel, channels
  constexpr int DYV = (P * TW * 4 + 255) / 256;
  uint4 dyr[DYV][WORDS];
  auto fetch_dy = [&](int j) {
#pragma unroll
    for (int u = 0; u < DYV; ++u) {
      const int e = tid + u * 256, p = e / (TW * 4), rem = e - p * (TW * 4);
      const int px = rem >> 2, cv = (rem & 3) * 8, oy = oy0 + j * P + p;
      const bool in = p < P && j * P + p < nrows && oy < OH && ox0 + px < OW && c0 + cv < C;
      const uint4* src = reinterpret_cast<const uint4*>(
          (const T*)g.dy + (in ? (obase + (size_t)oy * OW + ox0 + px) * C + c0 + cv : 0));
      dyr[u][0] = src[0];
      if constexpr (WORDS == 2) dyr[u][1] = src[1];
      if (!in) {
#pragma unroll
        for (int w = 0; w < WORDS; ++w) dyr[u][w] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto commit_dy = [&](int j) {
#pragma unroll
    for (int u = 0; u < DYV; ++u) {
      const int e = tid + u * 256, p = e / (TW * 4), rem = e - p * (TW * 4);
      if (p < P) {
        const int px = rem >> 2, cv = (rem & 3) * 8;
        float vals[8];
        unpack8(dyr[u], vals);
        float* d = &dys[WG ? (j & 1) : 0][(p * TW + px) * DCB + cv];
        reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
        reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
      }
    }
  };
  auto rows_of = [&](int j) { return j * P * S + K - S; };  // first new input row of step j

  // prologue: rows [0, NR) (+ dy rows) for step 0; step 1's in flight
  {
    DwRaw<NVP, WORDS> rp;
    fetch(rp, 0, NR);
    if constexpr (WG) fetch_dy(0);
    __syncthreads();  // xf / gt
    commit(rp, 0, NR);
    if constexpr (WG) commit_dy(0);
  }
  DwRaw<NVS, WORDS> rs;
  fetch(rs, rows_of(1), P * S);
  if constexpr (WG) fetch_dy(1);
  // PF = 2: a second register set keeps the step after next in flight too (steps alternate
  // between the sets; the loop is unrolled by two so both stay in registers)
  DwRaw<PF == 2 ? NVS : 1, WORDS> rs2;
  if constexpr (PF == 2) fetch(rs2, rows_of(2), P * S);
  __syncthreads();

  float s = 0.f, q = 0.f;                 // fwd BN statistics of channel c
  float acc[WG ? K * K : 1];              // wgrad taps of channel c
  if constexpr (WG) {
#pragma unroll
    for (int t = 0; t < K * K; ++t) acc[t] = 0.f;
  }
  auto store_step = [&](int j) {  // fwd output rows of step j from stage buffer j & 1 (after a barrier)
    for (int e = tid; e < P * TW * 4; e += 256) {
      const int p = e / (TW * 4), rem = e - p * (TW * 4);
      const int px = rem >> 2, cv = (rem & 3) * 8, oy = oy0 + j * P + p;
      if (j * P + p < nrows && ox0 + px < OW && c0 + cv < C) {
        T* dst = (T*)g.y + (obase + (size_t)oy * OW + ox0 + px) * C + c0 + cv;
        const T* src = &ost[WG ? 0 : (j & 1)][(p * TW + px) * DCB + cv];
        if constexpr (sizeof(T) == 2) {
          *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
        } else {
          reinterpret_cast<float4*>(dst)[0] = reinterpret_cast<const float4*>(src)[0];
          reinterpret_cast<float4*>(dst)[1] = reinterpret_cast<const float4*>(src)[1];
        }
      }
    }
  };
  auto step = [&](int j, auto& rsj) {
    if constexpr (!WG) {
      if (j > 0) store_step(j - 1);
    }
    if (j + 1 < nsteps) {  // rows of step j+1: ring slots and dy buffer step j does not read
      commit(rsj, rows_of(j + 1), P * S);
      if constexpr (WG) commit_dy(j + 1);
    }
    // unconditional: a conditional refill joins old and new values in a copy, and the copy
    // waits for the load (rows past the block are real or predicated-off elements)
    fetch(rsj, rows_of(j + 1 + PF), P * S);
    if constexpr (WG) fetch_dy(j + 2);
    int slot = (j * P * S) % R;
    if constexpr (!WG) {
      float o[P][CPG];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int t = 0; t < CPG; ++t) o[p][t] = 0.f;
#pragma unroll
      for (int ih = 0; ih < NR; ++ih) {  // input row ih feeds output row p through filter row ih - p*S
        const RT* rp = ringb + (slot * IWS + gc * CPG * S) * DCB + c;
        float win[WIN];
#pragma unroll
        for (int x = 0; x < WIN; ++x) {
          if constexpr (RB) win[x] = bf2f(rp[x * DCB]);
          else win[x] = rp[x * DCB];
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int kh = ih - p * S;
          if (kh < 0 || kh >= K) continue;
#pragma unroll
          for (int kw = 0; kw < K; ++kw)
#pragma unroll
            for (int t = 0; t < CPG; ++t) o[p][t] += win[t * S + kw] * wr[kh * K + kw];
        }
        slot = slot + 1 == R ? 0 : slot + 1;
      }
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const bool rowok = j * P + p < nrows;
#pragma unroll
        for (int t = 0; t < CPG; ++t) {
          const T ov = from_f<T>(o[p][t]);
          ost[j & 1][(p * TW + gc * CPG + t) * DCB + c] = ov;
          if (rowok && cvalid && ox0 + gc * CPG + t < OW) {
            s += o[p][t];
            q += o[p][t] * o[p][t];
            // the squeeze reads y as stored, as edet_se_squeeze would
            if constexpr (SQ) z += lazy_apply(to_f<T>(ov), ya, g.yv.act);
          }
        }
      }
    } else {
      float dv[P][CPG];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int t = 0; t < CPG; ++t) dv[p][t] = dys[j & 1][(p * TW + gc * CPG + t) * DCB + c];
#pragma unroll
      for (int ih = 0; ih < NR; ++ih) {
        const float* rp = ring + (slot * IWS + gc * CPG * S) * DCB + c;
        float win[WIN];
#pragma unroll
        for (int x = 0; x < WIN; ++x) win[x] = rp[x * DCB];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int kh = ih - p * S;
          if (kh < 0 || kh >= K) continue;
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            float a = 0.f;
#pragma unroll
            for (int t = 0; t < CPG; ++t) a += win[t * S + kw] * dv[p][t];
            acc[kh * K + kw] += a;
          }
        }
        slot = slot + 1 == R ? 0 : slot + 1;
      }
    }
    __syncthreads();
  };
  if constexpr (PF == 1) {
    for (int j = 0; j < nsteps; ++j) step(j, rs);
  } else {
    for (int j = 0; j < nsteps; j += 2) {
      step(j, rs);
      if (j + 1 < nsteps) step(j + 1, rs2);
    }
  }
  if constexpr (!WG) {
    store_step(nsteps - 1);
    if (g.has_stats) {  // the ring is free after the last barrier
      float* red = ring;
      red[gc * DCB + c] = s;
      red[(8 + gc) * DCB + c] = q;
      __syncthreads();
      if (tid < DCB && c0 + tid < C) {
        float ss = 0.f, qq = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) { ss += red[k * DCB + tid]; qq += red[(8 + k) * DCB + tid]; }
        stat_put(g.stats.sum[seg], c0 + tid, (double)ss);
        stat_put(g.stats.sq[seg], c0 + tid, (double)qq);
      }
    }
    if constexpr (SQ) {  // (after the statistics' reads of the scratch: its own rows 16..23)
      float* red = ring + 16 * DCB;
      red[gc * DCB + c] = z;
      __syncthreads();
      if (tid < DCB && c0 + tid < C) {
        float zz = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) zz += red[k * DCB + tid];
        atomicAdd(g.sq + (size_t)n * C + c0 + tid, (double)zz / (double)(OH * OW));
      }
    }
  } else {
    // column groups reduced one filter row at a time through the (free) ring: [K][8][32]
    float* red = ring;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
#pragma unroll
      for (int kw = 0; kw < K; ++kw) red[(kw * 8 + gc) * DCB + c] = acc[kh * K + kw];
      __syncthreads();
      if (tid < K * DCB) {
        const int kw = tid / DCB, cc = tid - kw * DCB;
        if (c0 + cc < C) {
          float sum = 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) sum += red[(kw * 8 + k) * DCB + cc];
          atomicAdd(g.dw + (size_t)(kh * K + kw) * C + c0 + cc, sum);
        }
      }
      __syncthreads();
    }
  }
}

template <typename T, int K, int S, int CPG, bool WG, int P>
static int launch_dws(DwArgs g, hipStream_t s) {
  constexpr int TW = 8 * CPG;
  int ohmax = 0;
  for (int i = 0; i < g.pout.nseg; ++i) ohmax = std::max(ohmax, g.pout.H[i]);
  DwsPlan pl{};
  long total = 0;
  // block target per shape (kbench sweep 512 / 1024 / 2048 over the D0 step): half the blocks
  // (longer strips) for the 32 x 32 layers and the BiFPN C = 64 filter gradients (32768 x 64
  // wgrad: 18.1 -> 12.8 us, 32768 x 672 k5 fwd: 57.8 -> 52.8 us), twice for the 128 x 128 k3
  // forward (148.6 -> 136.0 us)
  long rows_in = 0;
  for (int i = 0; i < g.pin.nseg; ++i) rows_in += (long)g.pin.batch * g.pin.H[i] * g.pin.W[i];
  int target = DWS_BLOCKS;
  if (WG) {
    if (g.C <= 64 || rows_in <= 32768) target = DWS_BLOCKS / 2;
  } else {
    if (rows_in <= 32768 && g.C >= 256) target = DWS_BLOCKS / 2;
    else if (K == 3 && S == 1 && rows_in >= 524288) target = 2 * DWS_BLOCKS;
    // the 256^2 stride-2 k3 forward: 4096 blocks (151.3 -> 140.8 us per step,
    // profiles/r03af_launch_size_sweep.txt)
    else if (S == 2 && rows_in >= 2097152) target = 4 * DWS_BLOCKS;
  }
  if (dev_knob(6) > 0) target = dev_knob(6);
  // rows per block: the most that still leaves >= target blocks, at least 2
  for (int TH = 256; TH >= 2; TH /= 2) {
    if (TH > 2 * ohmax && TH > 2) continue;
    total = 0;
    for (int i = 0; i < g.pout.nseg; ++i) {
      pl.strips[i] = cdiv(g.pout.W[i], TW);
      pl.rowblk[i] = cdiv(g.pout.H[i], TH);
      pl.nblk[i] = g.ncb * g.pout.batch * pl.rowblk[i] * pl.strips[i];
      total += pl.nblk[i];
    }
    pl.TH = TH;
    if (total >= target) break;
  }
  if (total == 0) return EDET_OK;
  pl.cb_inner = dev_knob(15) != 2;
  EDET_REQUIRE(total < (1L << 31), "dwconv: grid too large");
  if constexpr (!WG) {
    if (g.sq) {
      EDET_LAUNCH((k_dws<T, K, S, CPG, false, P, 1, false, true>), dim3((unsigned)total), dim3(256), 0, s, g, pl);
      return check_launch("edet dwconv (rows, squeeze)");
    }
  }
  // forward: two steps in flight (dw_bwd_probe r03o: 488 -> 480 us over the D0 stride-1 layers;
  // development slot 18 = 1 selects one)
  if (!WG && dev_knob(18) != 1) {
    EDET_LAUNCH((k_dws<T, K, S, CPG, false, P, 2>), dim3((unsigned)total), dim3(256), 0, s, g, pl);
    return check_launch("edet dwconv (rows)");
  }
  if constexpr (!WG && sizeof(T) == 2) {
    if (dev_knob(19) == 1) {  // development: bf16 ring
      EDET_LAUNCH((k_dws<T, K, S, CPG, false, P, 1, true>), dim3((unsigned)total), dim3(256), 0, s, g, pl);
      return check_launch("edet dwconv (rows)");
    }
  }
  EDET_LAUNCH((k_dws<T, K, S, CPG, WG, P>), dim3((unsigned)total), dim3(256), 0, s, g, pl);
  return check_launch("edet dwconv (rows)");
}

// strip width from the widest output segment: 32 columns where it fills them (16 at stride 2,
// whose input window is twice as wide; 8 or 32 columns there measured slower, as did 16 at
// stride 1)
template <typename T, int K, int S, bool WG>
static int dispatch_dws(const DwArgs& g, hipStream_t s) {
  int owmax = 0;
  for (int i = 0; i < g.pout.nseg; ++i) owmax = std::max(owmax, g.pout.W[i]);
  // two output rows per step at stride 1 (dw_sweep: fwd 991 -> 975, wgrad even; at stride 2
  // the ring would grow to K + 3S rows for little shared input)
  constexpr int P = S == 1 ? 2 : 1;
  if constexpr (S == 1) {
    if (owmax >= 32) return launch_dws<T, K, S, 4, WG, P>(g, s);
  }
  if (owmax >= 16) return launch_dws<T, K, S, 2, WG, P>(g, s);
  return launch_dws<T, K, S, 1, WG, P>(g, s);
}


// ------------------------------------------------------------------ fused backward (stride 1)
// One pass over dy and the lazy input x gives all three results of a stride-1 depthwise
// layer's backward, which the separate entry points compute in three passes (the transposed
// stencil and the filter gradient each read dy, and the BN-backward reduce of x's BatchNorm
// reads dx and x again, layers/mb_conv_block.py:144-154):
//   dx[r][c]   = sum_{kh,kw} dy[r+p-kh][c+p-kw] * w[kh][kw]              (p = (K-1)/2)
//   dW[kh][kw] += sum_{r,c} dy[r][c] * v(x)[r-p+kh][c-p+kw]
//   fold (optional): dbeta += sum du, dgamma += sum du * xhat with du = dx * act'(bn(x)):
//     edet_lazy_bwd_reduce over (x, dv = dx) without its own pass over HBM.
// Block = image x 32 channels x a strip of TW = 8*CPG columns x TH rows (channel block
// innermost, as in k_dws).  At stride 1 both results of row r read the same K rows of dy and
// v around r with the same column halo p, so the block walks down its rows keeping the last K
// of each in an LDS ring (dy in storage precision, exact; v transformed once, fp32); the next
// row is in flight in registers; one barrier per row.  Thread (c, gc) owns channel c and
// columns gc*CPG..: dx leaves as direct stores, the filter-gradient taps and the fold sums stay
// in registers until the block ends.
template <typename T, int K, int CPG, bool FOLD, int PF>
__global__ __launch_bounds__(256) void k_dwb(DwArgs g, DwsPlan pl, edet_bngrad64 fold) {
  constexpr int P = (K - 1) / 2;
  constexpr int TW = 8 * CPG, IWS = TW + K - 1;
  constexpr int R = K + 1;                      // ring rows: the K in use + the one committed
  constexpr int RV = IWS * (DCB / 8);           // 8-channel vectors per row and ring
  constexpr int WORDS = sizeof(T) == 2 ? 1 : 2;
  constexpr int WIN = CPG + K - 1;
  constexpr int RINGF = R * IWS * DCB;                     // v ring (floats)
  constexpr int RINGB = RINGF * 4 + R * IWS * DCB * (int)sizeof(T);  // + dy ring
  constexpr int REDB = (K * K + 2) * 8 * DCB * 4;          // end-of-block reductions
  constexpr int LDSB = RINGB > REDB ? RINGB : REDB;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  float* vring = reinterpret_cast<float*>(smem);
  T* dring = reinterpret_cast<T*>(smem + RINGF * 4);
  __shared__ float2 xf[DCB];
  __shared__ float gt[DCB];
  const int tid = threadIdx.x, c = tid & 31, gc = tid >> 5;

  int id = xcd_remap(blockIdx.x, gridDim.x), seg = 0;
  while (seg < g.pout.nseg - 1 && id >= pl.nblk[seg]) id -= pl.nblk[seg++];
  const int cb = id % g.ncb;
  id /= g.ncb;
  const int strip = id % pl.strips[seg];
  id /= pl.strips[seg];
  const int rb = id % pl.rowblk[seg];
  const int n = id / pl.rowblk[seg];
  const int c0 = cb * DCB, C = g.C;
  const int H = g.pin.H[seg], W = g.pin.W[seg];  // = the output's (stride 1)
  const int r0 = rb * pl.TH, x0 = strip * TW;
  const int nrows = min(pl.TH, H - r0);
  const T* X = (const T*)g.x + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * g.lz.ld + c0;
  const T* DY = (const T*)g.dy + ((size_t)g.pout.row_off[seg] + (size_t)n * H * W) * C + c0;
  T* DX = (T*)g.dx + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * C + c0;
  const bool cvalid = c0 + c < C;

  float wr[K * K];
  load_taps(wr, (const T*)g.w, C, c0 + c, cvalid);
  const float inv = 1.f / (float)seg_rows(g.pin, seg);
  if (tid < DCB) {
    const int cc = c0 + tid;
    xf[tid] = cc < C ? bn_affine(g.lz.bn, seg, cc, inv) : make_float2(1.f, 0.f);
    gt[tid] = (g.lz.gate && cc < C) ? g.lz.gate[(size_t)n * C + cc] : 1.f;
  }
  // the fold's per-channel constants of this thread's channel
  float2 myaf = make_float2(1.f, 0.f), mymr = make_float2(0.f, 1.f);
  if constexpr (FOLD) {
    if (cvalid) {
      myaf = bn_affine(g.lz.bn, seg, c0 + c, inv);
      mymr = bn_mean_rstd(g.lz.bn, seg, c0 + c, inv);
    }
  }

  // ring row t <-> image row q = r0 - P + t.  Each row is RV dy vectors and RV x vectors; dy
  // vector e of a fetch goes to thread e, x vector e to thread 255 - e (two uniform loops: one
  // loop over both with a per-lane choice held both paths' registers, ~190 VGPRs at k5)
  auto fetch = [&](auto& rg, auto& rx, int t0, int nt) {
    constexpr int NV = std::remove_reference_t<decltype(rg)>::NV;
    rg.ok = 0;
    rx.ok = 0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int v = (side ? 255 - tid : tid) + u * 256;
        const int row = v / RV, e = v - row * RV, xx = e >> 2, cv = (e & 3) * 8;
        const int q = r0 - P + t0 + row, gx = x0 - P + xx;
        const bool in = row < nt && q >= 0 && q < H && gx >= 0 && gx < W && c0 + cv < C;
        const uint32_t pix = in ? (uint32_t)(q * W + gx) : 0u;
        const uint4* src = reinterpret_cast<const uint4*>(side ? X + (size_t)pix * g.lz.ld + (in ? cv : 0)
                                                               : DY + (size_t)pix * C + (in ? cv : 0));
        auto& dst = side ? rx : rg;
        dst.v[u][0] = src[0];
        if constexpr (WORDS == 2) dst.v[u][1] = src[1];
        dst.ok |= (uint32_t)in << u;
      }
    }
  };
  auto commit = [&](const auto& rg, const auto& rx, int t0, int nt) {
    constexpr int NV = std::remove_reference_t<decltype(rg)>::NV;
#pragma unroll
    for (int u = 0; u < NV; ++u) {  // dy: copied as stored (zero outside the image)
      const int v = tid + u * 256;
      const int row = v / RV, e = v - row * RV, xx = e >> 2;
      if (row >= nt) break;
      const bool in = (rg.ok >> u) & 1;
      T* d = dring + (((t0 + row) % R) * IWS + xx) * DCB + (e & 3) * 8;
#pragma unroll
      for (int w = 0; w < WORDS; ++w) reinterpret_cast<uint4*>(d)[w] = in ? rg.v[u][w] : make_uint4(0, 0, 0, 0);
    }
    const int cv0 = ((255 - tid) & 3) * 8;  // this thread's 8 x channels, the same for every u
    float2 a8[8];
    float g8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a8[j] = xf[cv0 + j]; g8[j] = gt[cv0 + j]; }
    const int act = g.lz.act;
#pragma unroll
    for (int u = 0; u < NV; ++u) {  // x: transformed once (lazy BN / act / gate), fp32
      const int v = 255 - tid + u * 256;
      const int row = v / RV, e = v - row * RV, xx = e >> 2;
      if (row >= nt) break;
      float vals[8];
      if constexpr (WORDS == 1) {
        const uint32_t w4[4] = {rx.v[u][0].x, rx.v[u][0].y, rx.v[u][0].z, rx.v[u][0].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          vals[2 * i] = __uint_as_float(w4[i] << 16);
          vals[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
        }
      } else {
        const uint32_t w8[8] = {rx.v[u][0].x, rx.v[u][0].y, rx.v[u][0].z, rx.v[u][0].w,
                                rx.v[u][1].x, rx.v[u][1].y, rx.v[u][1].z, rx.v[u][1].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) vals[i] = __uint_as_float(w8[i]);
      }
      // transform unconditionally, zero the padding by a multiply (see k_dws commit)
      const float m = ((rx.ok >> u) & 1) ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = lazy_apply(vals[j], a8[j], act) * (g8[j] * m);
      float* d = vring + (((t0 + row) % R) * IWS + xx) * DCB + cv0;
      reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
      reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
    }
  };

  constexpr int NVS = (RV + 255) / 256;  // per thread and side, one row
  constexpr int NV2 = (2 * RV + 255) / 256;
  DwRaw<NVS, WORDS> rs, rsx;
  {
    // prologue rows two at a time (all K-1 at once held ~20 more VGPRs for the whole kernel)
    DwRaw<NV2, WORDS> rp, rpx;
    fetch(rp, rpx, 0, K - 1 < 2 ? K - 1 : 2);
    __syncthreads();  // xf / gt
#pragma unroll
    for (int t = 0; t < K - 1; t += 2) {
      commit(rp, rpx, t, K - 1 - t < 2 ? K - 1 - t : 2);
      if (t + 2 < K - 1) fetch(rp, rpx, t + 2, K - 1 - (t + 2) < 2 ? K - 1 - (t + 2) : 2);
    }
  }
  fetch(rs, rsx, K - 1, 1);
  // PF = 2: a second register set keeps the row after next in flight too (rows alternate
  // between the sets; the loop is unrolled by two so both stay in registers)
  DwRaw<PF == 2 ? NVS : 1, WORDS> rs2, rsx2;
  if constexpr (PF == 2) fetch(rs2, rsx2, K, 1);

  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  float fs = 0.f, fq = 0.f;
  const int act = g.lz.act;
  auto row_step = [&](int j, auto& rg, auto& rx) {
    const int r = r0 + j;
    // this row's global reads (the fold's x, read K-1 rows ago and cache-hot; dx for an
    // accumulating store) go out before the next row's prefetch: a load issued after it
    // would make its consumer wait for the prefetch too (vmcnt counts in issue order)
    T xr[CPG], dold[CPG];
    if constexpr (FOLD) {
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const int col = x0 + gc * CPG + i;
        const bool ok = col < W && cvalid;
        xr[i] = X[ok ? (size_t)(r * W + col) * g.lz.ld + c : 0];
      }
    }
    if (g.accumulate) {
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const int col = x0 + gc * CPG + i;
        const bool ok = col < W && cvalid;
        dold[i] = DX[ok ? (size_t)(r * W + col) * C + c : 0];
      }
    }
    commit(rg, rx, j + K - 1, 1);
    // unconditional refill (rows past the block are real or predicated-off elements)
    fetch(rg, rx, j + K - 1 + PF, 1);
    __syncthreads();

    float dxv[CPG], dyc[CPG];
#pragma unroll
    for (int i = 0; i < CPG; ++i) {
      dxv[i] = 0.f;
      dyc[i] = to_f<T>(dring[(((j + P) % R) * IWS + gc * CPG + i + P) * DCB + c]);
    }
#pragma unroll
    for (int rr = 0; rr < K; ++rr) {
      const int slot = (j + rr) % R;
      float dwin[WIN], vwin[WIN];
#pragma unroll
      for (int x = 0; x < WIN; ++x) {
        dwin[x] = to_f<T>(dring[(slot * IWS + gc * CPG + x) * DCB + c]);
        vwin[x] = vring[(slot * IWS + gc * CPG + x) * DCB + c];
      }
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const float wv = wr[(K - 1 - rr) * K + kw];
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < CPG; ++i) {
          dxv[i] += dwin[i + 2 * P - kw] * wv;
          a += dyc[i] * vwin[i + kw];
        }
        acc[rr * K + kw] += a;
      }
      // one ring row's windows live at a time (hoisting all K rows' LDS reads took the k5
      // forms to ~190 VGPRs, 2 waves per SIMD)
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < CPG; ++i) {
      const int col = x0 + gc * CPG + i;
      if (col < W && cvalid) {
        const T st = from_f<T>(g.accumulate ? to_f<T>(dold[i]) + dxv[i] : dxv[i]);
        DX[(size_t)(r * W + col) * C + c] = st;
        if constexpr (FOLD) {  // from the stored dx (the apply pass reads that value)
          const float xv = to_f<T>(xr[i]), yv = to_f<T>(st);
          const float du = act ? yv * dswishf_(xv * myaf.x + myaf.y) : yv;
          fs += du;
          fq += du * ((xv - mymr.x) * mymr.y);
        }
      }
    }
  };
  if constexpr (PF == 1) {
    for (int j = 0; j < nrows; ++j) row_step(j, rs, rsx);
  } else {
    for (int j = 0; j < nrows; j += 2) {
      row_step(j, rs, rsx);
      if (j + 1 < nrows) row_step(j + 1, rs2, rsx2);
    }
  }
  // block reductions over the 8 column groups: filter taps (+ fold sums), one atomic each
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < K * K; ++i) red[(i * 8 + gc) * DCB + c] = acc[i];
  if constexpr (FOLD) {
    red[(K * K * 8 + gc) * DCB + c] = fs;
    red[((K * K + 1) * 8 + gc) * DCB + c] = fq;
  }
  __syncthreads();
  constexpr int NOUT = (K * K + (FOLD ? 2 : 0)) * DCB;
  for (int e = tid; e < NOUT; e += 256) {
    const int i = e / DCB, cc = e - i * DCB;
    if (c0 + cc >= C) continue;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += red[(i * 8 + k) * DCB + cc];
    if (i < K * K) atomicAdd(g.dw + (size_t)i * C + c0 + cc, sum);
    else if constexpr (FOLD) stat_put(i == K * K ? fold.dbeta[seg] : fold.dgamma[seg], c0 + cc, (double)sum);
  }
}

// k_dwb with two output rows per step: every ring row's windows are read from LDS once for both
// rows (K + 1 ring rows feed 2 outputs instead of K feeding 1), and one barrier serves both.
// Ring R = K + 3: step j commits rows j+K-1, j+K into the slots of rows j-4, j-3, last read by
// step j-4, which step j-2's barrier separates from these writes.
template <typename T, int K, int CPG, bool FOLD>
__global__ __launch_bounds__(256) void k_dwb2(DwArgs g, DwsPlan pl, edet_bngrad64 fold) {
  constexpr int P = (K - 1) / 2;
  constexpr int TW = 8 * CPG, IWS = TW + K - 1;
  constexpr int R = K + 3;
  constexpr int RV = IWS * (DCB / 8);
  constexpr int WORDS = sizeof(T) == 2 ? 1 : 2;
  constexpr int WIN = CPG + K - 1;
  constexpr int RINGF = R * IWS * DCB;
  constexpr int RINGB = RINGF * 4 + R * IWS * DCB * (int)sizeof(T);
  constexpr int REDB = (K * K + 2) * 8 * DCB * 4;
  constexpr int LDSB = RINGB > REDB ? RINGB : REDB;
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  float* vring = reinterpret_cast<float*>(smem);
  T* dring = reinterpret_cast<T*>(smem + RINGF * 4);
  __shared__ float2 xf[DCB];
  __shared__ float gt[DCB];
  const int tid = threadIdx.x, c = tid & 31, gc = tid >> 5;

  int id = xcd_remap(blockIdx.x, gridDim.x), seg = 0;
  while (seg < g.pout.nseg - 1 && id >= pl.nblk[seg]) id -= pl.nblk[seg++];
  const int cb = id % g.ncb;
  id /= g.ncb;
  const int strip = id % pl.strips[seg];
  id /= pl.strips[seg];
  const int rb = id % pl.rowblk[seg];
  const int n = id / pl.rowblk[seg];
  const int c0 = cb * DCB, C = g.C;
  const int H = g.pin.H[seg], W = g.pin.W[seg];
  const int r0 = rb * pl.TH, x0 = strip * TW;
  const int nrows = min(pl.TH, H - r0);
  const T* X = (const T*)g.x + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * g.lz.ld + c0;
  const T* DY = (const T*)g.dy + ((size_t)g.pout.row_off[seg] + (size_t)n * H * W) * C + c0;
  T* DX = (T*)g.dx + ((size_t)g.pin.row_off[seg] + (size_t)n * H * W) * C + c0;
  const bool cvalid = c0 + c < C;

  float wr[K * K];
  load_taps(wr, (const T*)g.w, C, c0 + c, cvalid);
  const float inv = 1.f / (float)seg_rows(g.pin, seg);
  if (tid < DCB) {
    const int cc = c0 + tid;
    xf[tid] = cc < C ? bn_affine(g.lz.bn, seg, cc, inv) : make_float2(1.f, 0.f);
    gt[tid] = (g.lz.gate && cc < C) ? g.lz.gate[(size_t)n * C + cc] : 1.f;
  }
  float2 myaf = make_float2(1.f, 0.f), mymr = make_float2(0.f, 1.f);
  if constexpr (FOLD) {
    if (cvalid) {
      myaf = bn_affine(g.lz.bn, seg, c0 + c, inv);
      mymr = bn_mean_rstd(g.lz.bn, seg, c0 + c, inv);
    }
  }

  // as k_dwb: dy vector e of a fetch -> thread e, x vector e -> thread 255 - e
  auto fetch = [&](auto& rg, auto& rx, int t0, int nt) {
    constexpr int NV = std::remove_reference_t<decltype(rg)>::NV;
    rg.ok = 0;
    rx.ok = 0;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int v = (side ? 255 - tid : tid) + u * 256;
        const int row = v / RV, e = v - row * RV, xx = e >> 2, cv = (e & 3) * 8;
        const int q = r0 - P + t0 + row, gx = x0 - P + xx;
        const bool in = row < nt && q >= 0 && q < H && gx >= 0 && gx < W && c0 + cv < C;
        const uint32_t pix = in ? (uint32_t)(q * W + gx) : 0u;
        const uint4* src = reinterpret_cast<const uint4*>(side ? X + (size_t)pix * g.lz.ld + (in ? cv : 0)
                                                               : DY + (size_t)pix * C + (in ? cv : 0));
        auto& dst = side ? rx : rg;
        dst.v[u][0] = src[0];
        if constexpr (WORDS == 2) dst.v[u][1] = src[1];
        dst.ok |= (uint32_t)in << u;
      }
    }
  };
  auto commit = [&](const auto& rg, const auto& rx, int t0, int nt) {
    constexpr int NV = std::remove_reference_t<decltype(rg)>::NV;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = tid + u * 256;
      const int row = v / RV, e = v - row * RV, xx = e >> 2;
      if (row >= nt) break;
      const bool in = (rg.ok >> u) & 1;
      T* d = dring + (((t0 + row) % R) * IWS + xx) * DCB + (e & 3) * 8;
#pragma unroll
      for (int w = 0; w < WORDS; ++w) reinterpret_cast<uint4*>(d)[w] = in ? rg.v[u][w] : make_uint4(0, 0, 0, 0);
    }
    const int cv0 = ((255 - tid) & 3) * 8;
    float2 a8[8];
    float g8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a8[j] = xf[cv0 + j]; g8[j] = gt[cv0 + j]; }
    const int act = g.lz.act;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int v = 255 - tid + u * 256;
      const int row = v / RV, e = v - row * RV, xx = e >> 2;
      if (row >= nt) break;
      float vals[8];
      if constexpr (WORDS == 1) {
        const uint32_t w4[4] = {rx.v[u][0].x, rx.v[u][0].y, rx.v[u][0].z, rx.v[u][0].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          vals[2 * i] = __uint_as_float(w4[i] << 16);
          vals[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
        }
      } else {
        const uint32_t w8[8] = {rx.v[u][0].x, rx.v[u][0].y, rx.v[u][0].z, rx.v[u][0].w,
                                rx.v[u][1].x, rx.v[u][1].y, rx.v[u][1].z, rx.v[u][1].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) vals[i] = __uint_as_float(w8[i]);
      }
      const float m = ((rx.ok >> u) & 1) ? 1.f : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) vals[j] = lazy_apply(vals[j], a8[j], act) * (g8[j] * m);
      float* d = vring + (((t0 + row) % R) * IWS + xx) * DCB + cv0;
      reinterpret_cast<float4*>(d)[0] = make_float4(vals[0], vals[1], vals[2], vals[3]);
      reinterpret_cast<float4*>(d)[1] = make_float4(vals[4], vals[5], vals[6], vals[7]);
    }
  };

  constexpr int NV2 = (2 * RV + 255) / 256;
  DwRaw<NV2, WORDS> rs, rsx;
  {  // prologue: rows 0 .. K-2, two at a time
    DwRaw<NV2, WORDS> rp, rpx;
    fetch(rp, rpx, 0, K - 1 < 2 ? K - 1 : 2);
    __syncthreads();  // xf / gt
#pragma unroll
    for (int t = 0; t < K - 1; t += 2) {
      commit(rp, rpx, t, K - 1 - t < 2 ? K - 1 - t : 2);
      if (t + 2 < K - 1) fetch(rp, rpx, t + 2, K - 1 - (t + 2) < 2 ? K - 1 - (t + 2) : 2);
    }
  }
  fetch(rs, rsx, K - 1, 2);

  float acc[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) acc[i] = 0.f;
  float fs = 0.f, fq = 0.f;
  const int act = g.lz.act;
  for (int j = 0; j < nrows; j += 2) {
    // this step's global reads (fold x of both rows, cache-hot; dx for an accumulating store)
    // before the next rows' prefetch (vmcnt counts in issue order)
    T xr[2][CPG], dold[2][CPG];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const int col = x0 + gc * CPG + i, r = r0 + j + p;
        const bool ok = col < W && cvalid && j + p < nrows;
        if constexpr (FOLD) xr[p][i] = X[ok ? (size_t)(r * W + col) * g.lz.ld + c : 0];
        if (g.accumulate) dold[p][i] = DX[ok ? (size_t)(r * W + col) * C + c : 0];
      }
    commit(rs, rsx, j + K - 1, 2);
    fetch(rs, rsx, j + K + 1, 2);  // unconditional (rows past the block: real or predicated off)
    __syncthreads();

    float dxv[2][CPG], dyc[2][CPG];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        dxv[p][i] = 0.f;
        // an odd block's last step has no second row: its dy (a real row of the next block or
        // padding) must not reach the filter gradient
        const float live = j + p < nrows ? 1.f : 0.f;
        dyc[p][i] = to_f<T>(dring[(((j + p + P) % R) * IWS + gc * CPG + i + P) * DCB + c]) * live;
      }
#pragma unroll
    for (int rr = 0; rr <= K; ++rr) {
      const int slot = (j + rr) % R;
      float dwin[WIN], vwin[WIN];
#pragma unroll
      for (int x = 0; x < WIN; ++x) {
        dwin[x] = to_f<T>(dring[(slot * IWS + gc * CPG + x) * DCB + c]);
        vwin[x] = vring[(slot * IWS + gc * CPG + x) * DCB + c];
      }
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int kh = rr - p;
        if (kh < 0 || kh >= K) continue;
#pragma unroll
        for (int kw = 0; kw < K; ++kw) {
          const float wv = wr[(K - 1 - kh) * K + kw];
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < CPG; ++i) {
            dxv[p][i] += dwin[i + 2 * P - kw] * wv;
            a += dyc[p][i] * vwin[i + kw];
          }
          acc[kh * K + kw] += a;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < CPG; ++i) {
        const int col = x0 + gc * CPG + i, r = r0 + j + p;
        if (col < W && cvalid && j + p < nrows) {
          const T st = from_f<T>(g.accumulate ? to_f<T>(dold[p][i]) + dxv[p][i] : dxv[p][i]);
          DX[(size_t)(r * W + col) * C + c] = st;
          if constexpr (FOLD) {  // from the stored dx (the apply pass reads that value)
            const float xv = to_f<T>(xr[p][i]), yv = to_f<T>(st);
            const float du = act ? yv * dswishf_(xv * myaf.x + myaf.y) : yv;
            fs += du;
            fq += du * ((xv - mymr.x) * mymr.y);
          }
        }
      }
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < K * K; ++i) red[(i * 8 + gc) * DCB + c] = acc[i];
  if constexpr (FOLD) {
    red[(K * K * 8 + gc) * DCB + c] = fs;
    red[((K * K + 1) * 8 + gc) * DCB + c] = fq;
  }
  __syncthreads();
  constexpr int NOUT = (K * K + (FOLD ? 2 : 0)) * DCB;
  for (int e = tid; e < NOUT; e += 256) {
    const int i = e / DCB, cc = e - i * DCB;
    if (c0 + cc >= C) continue;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += red[(i * 8 + k) * DCB + cc];
    if (i < K * K) atomicAdd(g.dw + (size_t)i * C + c0 + cc, sum);
    else if constexpr (FOLD) stat_put(i == K * K ? fold.dbeta[seg] : fold.dgamma[seg], c0 + cc, (double)sum);
  }
}

// ------------------------------------------------------------------ tiled fused backward (stride 1)
// The same three results as k_dwb (dx, the filter gradient, the input BN's backward sums) with
// no row-serial ring: a block owns one image x 16 channels and walks `tpb` 16 x 16 pixel tiles.
// Per tile every dy and x vector of the (16 + K - 1)^2 halo window is requested at once (all in
// flight together), dy is parked in LDS as stored and v(x) = act(bn(x)) * gate once in fp32,
// then thread (channel c, patch row pr, wave = patch column) computes a 4 x 4 pixel patch of its
// channel straight from LDS: dx from the dy window (the channel's K*K taps in registers), the
// filter gradient from the v window against the patch's own dy (accumulated in registers over
// all the block's tiles), both from the same (K + 3) x (K + 3) window rows.  dx goes back through
// LDS and leaves as 16-byte vectors.  Two barriers per tile instead of one per output row: the
// 32 x 32 and 16 x 16 planes of the late MBConv stages (where k_dwb's rings hold a handful of
// rows per block and wait on memory between them) become a few fully overlapped load rounds.
// LDS rows are padded so a wave's four patch rows (4 image rows apart) fall in disjoint banks.
constexpr int DWT_T = 16;   // tile edge
constexpr int DWT_CB = 16;  // channels per block

struct DwtPlan {
  int ntx[EDET_MAX_SEG];     // tiles across an image
  int ntiles[EDET_MAX_SEG];  // tiles per image
  int chunks[EDET_MAX_SEG];  // chunks of tpb consecutive (image, tile) tiles per segment (GIN: per image)
  int nblk[EDET_MAX_SEG];    // blocks of the segment: batch * chunks * ncg
  int tpb, ncg;
};

// GIN (edet_dwconv_bwd_lazy): g.dy is not d(raw y) but the lazy gradient g.dyl -- dv, the
// value's raw y and its BN-backward tables -- and the dy window is built on load with
// edet_lazy_bwd_apply's formula (d(raw y) = sc*du + kb*y + kc, du = (dv*gate + dsq)*act'(bn(y))),
// rounded to T as that pass would store it: the apply's pass over (dv, y) and the write and
// re-read of d(raw y) are gone (one extra y stream here instead)
template <typename T, int K, bool FOLD, bool GIN = false>
__global__ __launch_bounds__(256) void k_dwt(DwArgs g, DwtPlan pl, edet_bngrad64 fold) {
  constexpr int P = (K - 1) / 2, IT = DWT_T + K - 1, NPX = IT * IT;
  constexpr int EPV = 16 / (int)sizeof(T);  // elements per 16-byte vector
  constexpr int VPP = DWT_CB / EPV;         // vectors per pixel (16 channels)
  constexpr int NV = NPX * VPP, NL = (NV + 255) / 256;
  constexpr int KK = K * K;
  // padded row strides (elements): 4 rows apart land 16 (dy bf16: 8) dwords apart in the banks
  constexpr int DRS = IT * DWT_CB + (sizeof(T) == 2 ? 8 : 4), VRS = IT * DWT_CB + 4;
  __shared__ __attribute__((aligned(16))) T dys[IT * DRS];       // dy window as stored; dx stage
  __shared__ __attribute__((aligned(16))) float vs[IT * VRS];    // v(x) window; reductions
  __shared__ __attribute__((aligned(16))) T xs[FOLD ? DWT_T * DWT_T * DWT_CB : 8];  // raw x, interior
  __shared__ float2 af[DWT_CB];
  __shared__ float gt[DWT_CB];
  __shared__ float4 gtab[GIN ? DWT_CB : 1];  // GIN: y's (sc, sh, kb, kc) per channel
  __shared__ float2 ggd[GIN ? DWT_CB : 1];   // GIN: (gate, dsq) of this image per channel
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  int id = xcd_remap(blockIdx.x, gridDim.x), seg = 0;
  while (seg < g.pin.nseg - 1 && id >= pl.nblk[seg]) id -= pl.nblk[seg++];
  const int cg = id % pl.ncg;
  id /= pl.ncg;
  // a chunk is tpb consecutive tiles of the segment's (image, tile) sequence: on the small
  // planes (one to four tiles per image) a block walks several images of its channel group
  // (GIN keeps one image per block: its per-image tables would cost the k5 fold form its
  // second wave per SIMD)
  const int chunk = GIN ? id % pl.chunks[seg] : id;
  const int n_gin = GIN ? id / pl.chunks[seg] : 0;
  const int c0 = cg * DWT_CB, C = g.C;
  const int H = g.pin.H[seg], W = g.pin.W[seg];
  const size_t HW = (size_t)H * W;
  const T* X0 = (const T*)g.x + (size_t)g.pin.row_off[seg] * g.lz.ld + c0;
  const T* DY0 = (const T*)(GIN ? g.dyl.dv : g.dy) + (size_t)g.pout.row_off[seg] * C + c0;
  const T* YR0 = GIN ? (const T*)g.dyl.y.x + (size_t)g.pout.row_off[seg] * C + c0 : nullptr;
  T* DX0 = (T*)g.dx + (size_t)g.pin.row_off[seg] * C + c0;
  const float inv = 1.f / (float)seg_rows(g.pin, seg);
  if (tid < DWT_CB) {
    af[tid] = bn_affine(g.lz.bn, seg, c0 + tid, inv);
    if constexpr (GIN) {
      // edet_lazy_bwd_apply's tables (bn.hip load_tables + the kb / kc fold), same arithmetic
      const edet_dgrad_lazy& d = g.dyl;
      const int cc = c0 + tid;
      float4 t = make_float4(1.f, 0.f, 0.f, 0.f);
      if (d.y.bn.enabled) {
        const float2 a = bn_affine(d.y.bn, seg, cc, inv), q = bn_mean_rstd(d.y.bn, seg, cc, inv);
        const float dgm = (float)(stat_get(d.acc.dgamma[seg], cc) * (double)inv),
                    dbm = (float)(stat_get(d.acc.dbeta[seg], cc) * (double)inv);
        const float kb = -a.x * q.y * dgm;
        t = make_float4(a.x, a.y, kb, -a.x * dbm - kb * q.x);
        // one writer per segment and channel: the first chunk's block
        if (n_gin == 0 && chunk == 0 && d.grads.a[seg]) {
          d.grads.a[seg][cc] += (float)stat_get(d.acc.dgamma[seg], cc);
          d.grads.b[seg][cc] += (float)stat_get(d.acc.dbeta[seg], cc);
        }
      }
      gtab[tid] = t;
      gt[tid] = g.lz.gate ? g.lz.gate[(size_t)n_gin * C + cc] : 1.f;
      ggd[tid] = make_float2(d.y.gate ? d.y.gate[(size_t)n_gin * C + cc] : 1.f,
                             d.dsq ? d.dsq[(size_t)n_gin * C + cc] : 0.f);
    }
  }
  // this thread: channel c, the 4 x 4 patch at rows a0 .., columns b0 .. of every tile
  const int c = lane & 15, a0 = (lane >> 4) * 4, b0 = wave * 4;
  float w[KK];
  load_taps(w, (const T*)g.w, C, c0 + c, true);
  float4 ft = make_float4(0.f, 0.f, 0.f, 1.f);  // fold: this channel's (scale, shift, mean, rstd)
  if constexpr (FOLD) {
    const float2 a = bn_affine(g.lz.bn, seg, c0 + c, inv), m = bn_mean_rstd(g.lz.bn, seg, c0 + c, inv);
    ft = make_float4(a.x, a.y, m.x, m.y);
  }
  float dwa[KK];
#pragma unroll
  for (int i = 0; i < KK; ++i) dwa[i] = 0.f;
  float fs = 0.f, fq = 0.f;
  const int act = g.lz.act;
  const int nt = pl.ntiles[seg];
  const int t_begin = chunk * pl.tpb, t_end = min((GIN ? 1 : g.pin.batch) * nt, t_begin + pl.tpb);
  int cur_n = -1;
  for (int t = t_begin; t < t_end; ++t) {
    const int n = GIN ? n_gin : t / nt, tl = GIN ? t : t - n * nt;
    const int y0 = (tl / pl.ntx[seg]) * DWT_T, x0 = (tl % pl.ntx[seg]) * DWT_T;
    const T* X = X0 + n * HW * g.lz.ld;
    const T* DY = DY0 + n * HW * C;
    const T* YR = GIN ? YR0 + n * HW * C : nullptr;
    T* DX = DX0 + n * HW * C;
    if constexpr (!GIN) {
      if (n != cur_n) {  // this image's SE gate (read in the commit, after the barrier below)
        cur_n = n;
        if (tid < DWT_CB) gt[tid] = g.lz.gate ? g.lz.gate[(size_t)n * C + c0 + tid] : 1.f;
      }
    }
    // ---- the halo window of dy and x: every vector requested before any is used
    uint4 rd[NL], rx[NL], ry[GIN ? NL : 1];
    uint32_t okm = 0;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int e = tid + u * 256, px = e / VPP, q = e - px * VPP;
      const int i = px / IT, j = px - i * IT, gy = y0 - P + i, gx = x0 - P + j;
      const bool ok = e < NV && gy >= 0 && gy < H && gx >= 0 && gx < W;
      const uint32_t pix = ok ? (uint32_t)(gy * W + gx) : 0u;
      const uint4 a = *reinterpret_cast<const uint4*>(DY + (size_t)pix * C + (ok ? q * EPV : 0));
      const uint4 b = *reinterpret_cast<const uint4*>(X + (size_t)pix * g.lz.ld + (ok ? q * EPV : 0));
      if constexpr (GIN) {
        ry[u] = *reinterpret_cast<const uint4*>(YR + (size_t)pix * C + (ok ? q * EPV : 0));
        rd[u] = a;  // zeroed after the transform (kc != 0 off the plane)
      } else {
        rd[u] = ok ? a : make_uint4(0, 0, 0, 0);
      }
      rx[u] = b;
      okm |= (uint32_t)ok << u;
    }
    __syncthreads();  // the previous tile's LDS reads are done (and the tables are in place)
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int e = tid + u * 256, px = e / VPP, q = e - px * VPP;
      if (e >= NV) break;
      const int i = px / IT, j = px - i * IT;
      const float m = ((okm >> u) & 1) ? 1.f : 0.f;  // zero padding of the transformed input
      if constexpr (GIN) {
        const T* de = reinterpret_cast<const T*>(&rd[u]);
        const T* ye = reinterpret_cast<const T*>(&ry[u]);
        const int yact = g.dyl.y.act;
        T o[EPV];
#pragma unroll
        for (int jj = 0; jj < EPV; ++jj) {
          const int cc = q * EPV + jj;
          const float4 tb = gtab[cc];
          const float2 gd = ggd[cc];
          const float yv = to_f<T>(ye[jj]);
          float gg = to_f<T>(de[jj]);
          gg *= gd.x;
          gg += gd.y;
          const float du = yact ? gg * dswishf_(yv * tb.x + tb.y) : gg;
          const float v = tb.x * du + tb.z * yv + tb.w;
          o[jj] = from_f<T>(v * m);
        }
        *reinterpret_cast<uint4*>(dys + i * DRS + j * DWT_CB + q * EPV) = *reinterpret_cast<const uint4*>(o);
      } else {
        *reinterpret_cast<uint4*>(dys + i * DRS + j * DWT_CB + q * EPV) = rd[u];
      }
      const T* xe = reinterpret_cast<const T*>(&rx[u]);
      float vals[EPV];
#pragma unroll
      for (int jj = 0; jj < EPV; ++jj) {
        const int cc = q * EPV + jj;
        vals[jj] = lazy_apply(to_f<T>(xe[jj]), af[cc], act) * (gt[cc] * m);
      }
#pragma unroll
      for (int jj = 0; jj < EPV; jj += 4)
        *reinterpret_cast<float4*>(vs + i * VRS + j * DWT_CB + q * EPV + jj) =
            make_float4(vals[jj], vals[jj + 1], vals[jj + 2], vals[jj + 3]);
      if constexpr (FOLD) {
        if (i >= P && i < P + DWT_T && j >= P && j < P + DWT_T)
          *reinterpret_cast<uint4*>(xs + ((i - P) * DWT_T + (j - P)) * DWT_CB + q * EPV) = rx[u];
      }
    }
    __syncthreads();
    // ---- the patch: dx from the dy window, the filter gradient from the v window.  The window
    // bases are made opaque per tile: otherwise every one of the ~(K+3)^2 LDS addresses is
    // hoisted out of the tile loop into a register of its own (~60 VGPRs); from one base each
    // read is an immediate offset
    int dofs = a0 * DRS + b0 * DWT_CB + c, vofs = a0 * VRS + b0 * DWT_CB + c;
    asm volatile("" : "+v"(dofs), "+v"(vofs));
    const T* db = dys + dofs;
    const float* vb = vs + vofs;
    float dyi[4][4], dxa[4][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        dyi[e][f] = to_f<T>(db[(e + P) * DRS + (f + P) * DWT_CB]);
        dxa[e][f] = 0.f;
      }
#pragma unroll
    for (int r = 0; r < K + 3; ++r) {
      float dyw[K + 3], vw[K + 3];
#pragma unroll
      for (int sc = 0; sc < K + 3; ++sc) {
        dyw[sc] = to_f<T>(db[r * DRS + sc * DWT_CB]);
        vw[sc] = vb[r * VRS + sc * DWT_CB];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kh = e + 2 * P - r;  // dx row a0+e takes dy window row r through tap row kh
        if (kh >= 0 && kh < K) {
#pragma unroll
          for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int kw = 0; kw < K; ++kw) dxa[e][f] += dyw[f + 2 * P - kw] * w[kh * K + kw];
        }
        const int kv = r - e;  // dW row kv takes v window row r against the dy of pixel row a0+e
        if (kv >= 0 && kv < K) {
#pragma unroll
          for (int kw = 0; kw < K; ++kw) {
            float a = 0.f;
#pragma unroll
            for (int f = 0; f < 4; ++f) a += dyi[e][f] * vw[f + kw];
            dwa[kv * K + kw] += a;
          }
        }
      }
      // (dx as v_pk_fma_f32 column pairs: the odd-aligned dy pairs need copies, 247 -> 300
      // registers at k5 fold (occupancy 2 -> 1), 155 -> 176 at k3 fold (3 -> 2); not kept.
      // No per-row pinning of the window or the taps: the SLP vectorizer then gathers the whole
      // filter gradient into v_pk_fma_f32 after the last row -- the full v window in registers,
      // ~210-250 VGPRs at k5, but half the FMA instructions; pinned rows with scalar FMAs held
      // 140 VGPRs and ran 5-10 % slower at k5, even at k3: tools/dwt_ab.py r04e-r04g)
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // every dy / v read is done: dys takes the dx tile [16][16][16]
    int sofs = (a0 * DWT_T + b0) * DWT_CB + c;  // (opaque per tile, as the window bases)
    asm volatile("" : "+v"(sofs));
    T* sb = dys + sofs;
    const T* xb = xs + (FOLD ? sofs : 0);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int po = (e * DWT_T + f) * DWT_CB;
        const T sv = from_f<T>(dxa[e][f]);
        sb[po] = sv;
        if constexpr (FOLD) {  // BN-backward sums of x's BatchNorm from the stored dx
          // branch-free: pixels past the plane edge (stale LDS) are selected out, not skipped
          const bool in = y0 + a0 + e < H && x0 + b0 + f < W;
          const float yv = to_f<T>(sv), xv = to_f<T>(xb[po]);
          const float du = act ? yv * dswishf_(xv * ft.x + ft.y) : yv;
          fs += in ? du : 0.f;
          fq += in ? du * ((xv - ft.z) * ft.w) : 0.f;
          asm volatile("" : "+v"(fs), "+v"(fq));  // pixel by pixel (no batched transcendentals)
        }
      }
    __syncthreads();
    // ---- dx tile out as 16-byte vectors (accumulate: read-add-write)
#pragma unroll
    for (int u = 0; u < VPP; ++u) {
      const int e = tid + u * 256, px = e / VPP, q = e - px * VPP;
      const int gy = y0 + px / DWT_T, gx = x0 + px % DWT_T;
      if (gy < H && gx < W) {
        T* dst = DX + (size_t)(gy * W + gx) * C + q * EPV;
        const uint4 v = *reinterpret_cast<const uint4*>(dys + px * DWT_CB + q * EPV);
        if (g.accumulate) {
          const T* ve = reinterpret_cast<const T*>(&v);
          const uint4 o4 = *reinterpret_cast<const uint4*>(dst);
          const T* oe = reinterpret_cast<const T*>(&o4);
          T o[EPV];
#pragma unroll
          for (int jj = 0; jj < EPV; ++jj) o[jj] = from_f<T>(to_f<T>(ve[jj]) + to_f<T>(oe[jj]));
          *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(o);
        } else {
          *reinterpret_cast<uint4*>(dst) = v;
        }
      }
    }
  }
  // ---- block reductions: over the wave's 4 patch rows (lane bits 4-5), then the 4 waves in LDS
  // in a fixed order; one fp32 atomic per (tap, channel), one fp64 atomic per fold sum and channel
#pragma unroll
  for (int i = 0; i < KK; ++i) {
    float v = dwa[i];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    dwa[i] = v;
  }
  if constexpr (FOLD) {
    fs += __shfl_xor(fs, 16, 64);
    fs += __shfl_xor(fs, 32, 64);
    fq += __shfl_xor(fq, 16, 64);
    fq += __shfl_xor(fq, 32, 64);
  }
  __syncthreads();  // vs is free: [4 waves][KK + 2][16]
  float* red = vs;
  constexpr int NR = KK + (FOLD ? 2 : 0);
  if (lane < 16) {
#pragma unroll
    for (int i = 0; i < KK; ++i) red[(wave * NR + i) * DWT_CB + c] = dwa[i];
    if constexpr (FOLD) {
      red[(wave * NR + KK) * DWT_CB + c] = fs;
      red[(wave * NR + KK + 1) * DWT_CB + c] = fq;
    }
  }
  __syncthreads();
  for (int e = tid; e < NR * DWT_CB; e += 256) {
    const int i = e / DWT_CB, cc = e - i * DWT_CB;
    const float v = (red[(0 * NR + i) * DWT_CB + cc] + red[(1 * NR + i) * DWT_CB + cc]) +
                    (red[(2 * NR + i) * DWT_CB + cc] + red[(3 * NR + i) * DWT_CB + cc]);
    if (i < KK) atomicAdd(g.dw + (size_t)i * C + c0 + cc, v);
    else if constexpr (FOLD) stat_put(i == KK ? fold.dbeta[seg] : fold.dgamma[seg], c0 + cc, (double)v);
  }
}

template <typename T, int K, bool FOLD, bool GIN = false>
static int launch_dwt(DwArgs g, const edet_bngrad64& fold, hipStream_t s) {
  DwtPlan pl{};
  pl.ncg = g.C / DWT_CB;
  long tiles = 0;
  for (int i = 0; i < g.pin.nseg; ++i) {
    pl.ntx[i] = cdiv(g.pin.W[i], DWT_T);
    pl.ntiles[i] = pl.ntx[i] * cdiv(g.pin.H[i], DWT_T);
    tiles += (long)g.pin.batch * pl.ntiles[i] * pl.ncg;
  }
  // tiles per block: the most (<= 8) that still leaves >= 768 blocks -- fewer filter-gradient
  // flushes and prologues per tile (tools/dwt_ab.py sweep r04e: 256^2 x 32 207 -> 178 us at 8,
  // 32^2 x 480 k5 82 -> 77 at 4; the C = 64 32^2 level wants all 512 blocks).  Development slots
  // 30 / 31: block floor / tiles per block
  int tpb = 1;
  // (round 6, r06ak: the five-level C = 64 head pyramids take the 384 floor, 235.5 -> 225.4 us
  // over their calls; every other shape keeps 768)
  const long floor_blocks = dev_knob(30) > 0 ? dev_knob(30) : (g.pin.nseg > 1 ? 384 : 768);
  while (tpb < 8 && tiles / (2 * tpb) >= floor_blocks) tpb *= 2;
  if (dev_knob(31) > 0) tpb = dev_knob(31);
  pl.tpb = tpb;
  long total = 0;
  for (int i = 0; i < g.pin.nseg; ++i) {
    // chunks span images (GIN: chunks of one image, per image)
    pl.chunks[i] = cdiv((GIN ? 1 : g.pin.batch) * pl.ntiles[i], tpb);
    pl.nblk[i] = (GIN ? g.pin.batch : 1) * pl.chunks[i] * pl.ncg;
    total += pl.nblk[i];
  }
  if (total == 0) return EDET_OK;
  EDET_REQUIRE(total < (1L << 31), "dwconv_bwd: grid too large");
  EDET_LAUNCH((k_dwt<T, K, FOLD, GIN>), dim3((unsigned)total), dim3(256), 0, s, g, pl, fold);
  return check_launch("edet dwconv bwd (tiles)");
}

template <typename T, int K, int CPG, bool FOLD>
static int launch_dwb(DwArgs g, const edet_bngrad64& fold, hipStream_t s) {
  // rows in flight ahead of the one committed (development slot 17 = 2 selects two)
  const int pf = dev_knob(17) == 2 ? 2 : 1;
  constexpr int TW = 8 * CPG;
  int hmax = 0;
  long rows_in = 0;
  for (int i = 0; i < g.pin.nseg; ++i) {
    hmax = std::max(hmax, g.pin.H[i]);
    rows_in += (long)g.pin.batch * g.pin.H[i] * g.pin.W[i];
  }
  // plan per shape (tools/dw_bwd_probe.py over the D0 b32 stride-1 layers, r03k): two output
  // rows per step (k_dwb2) everywhere but the C = 64 BiFPN / head layers (their short rows keep
  // the 1-row ring: 44 vs 45 us pyramid, 32 vs 35 us at 64^2); 512 blocks at k5 (C = 240 / 480:
  // 143 -> 138, 88 -> 78 us), 2048 for the large k3 layers (256^2 x 32: 191 -> 174, 128^2 x 144:
  // 220 -> 209 us).  Development slots: 16 = block target, 25 = rows per step (1 or 2)
  const int rows_per_step = dev_knob(25) ? dev_knob(25) : (g.C <= 64 ? 1 : 2);
  DwsPlan pl{};
  pl.cb_inner = 1;
  long total = 0;
  int target = DWS_BLOCKS;
  if (K == 5) target = DWS_BLOCKS / 2;
  else if (rows_in >= 524288) target = 2 * DWS_BLOCKS;
  // round 3 (profiles/r03af_launch_size_sweep.txt): the single-level BiFPN C = 64 layers and the
  // 32 x 32 k5 C = 480 layer want longer strips (32768 x 64: 116.7 -> 92.6 us per step at 512,
  // 8192 x 64: 71.6 -> 63.1 at 256, 32768 x 480 k5: 73.5 -> 69.3 at 256)
  if (g.C <= 64 && g.pin.nseg == 1 && rows_in <= 32768) target = rows_in <= 8192 ? 256 : 512;
  else if (K == 5 && g.C <= 480 && rows_in <= 32768) target = 256;
  if (dev_knob(16) > 0) target = dev_knob(16);
  for (int TH = 256; TH >= 2; TH /= 2) {
    if (TH > 2 * hmax && TH > 2) continue;
    total = 0;
    for (int i = 0; i < g.pin.nseg; ++i) {
      pl.strips[i] = cdiv(g.pin.W[i], TW);
      pl.rowblk[i] = cdiv(g.pin.H[i], TH);
      pl.nblk[i] = g.ncb * g.pin.batch * pl.rowblk[i] * pl.strips[i];
      total += pl.nblk[i];
    }
    pl.TH = TH;
    if (total >= target) break;
  }
  if (total == 0) return EDET_OK;
  EDET_REQUIRE(total < (1L << 31), "dwconv_bwd: grid too large");
  if (rows_per_step == 2) EDET_LAUNCH((k_dwb2<T, K, CPG, FOLD>), dim3((unsigned)total), dim3(256), 0, s, g, pl, fold);
  else if (pf == 2) EDET_LAUNCH((k_dwb<T, K, CPG, FOLD, 2>), dim3((unsigned)total), dim3(256), 0, s, g, pl, fold);
  else EDET_LAUNCH((k_dwb<T, K, CPG, FOLD, 1>), dim3((unsigned)total), dim3(256), 0, s, g, pl, fold);
  return check_launch("edet dwconv bwd");
}

template <typename T, int K, bool FOLD>
static int dispatch_dwb_cpg(const DwArgs& g, const edet_bngrad64& fold, hipStream_t s) {
  // the tiled form (k_dwt) for bf16 storage wherever it applies: 1068 -> 944 us over the D0 b32
  // shapes, no shape slower (tools/dwt_ab.py, r04h; 32^2 x 480 k5 even); fp32 (parity runs)
  // keeps the row-streaming kernels (tiles at 1-2 blocks per CU: 1185 vs 1205 us).
  // Development slot 29: 1 forces the tiled form, 2 the row-streaming kernels
  const int form = dev_knob(29);
  if (form != 2 && g.C % DWT_CB == 0 && g.lz.ld % 8 == 0 && (form == 1 || sizeof(T) == 2))
    return launch_dwt<T, K, FOLD>(g, fold, s);
  int wmax = 0;
  for (int i = 0; i < g.pin.nseg; ++i) wmax = std::max(wmax, g.pin.W[i]);
  const int force = dev_knob(20);  // development: columns per thread (1, 2, 4)
  if (force == 4 || (!force && wmax >= 32)) return launch_dwb<T, K, 4, FOLD>(g, fold, s);
  if (force == 2 || (!force && wmax >= 16)) return launch_dwb<T, K, 2, FOLD>(g, fold, s);
  return launch_dwb<T, K, 1, FOLD>(g, fold, s);
}

template <typename T>
static int dispatch_dwb(int k, const DwArgs& g, const edet_bngrad64* fold, hipStream_t s) {
  const edet_bngrad64 f = fold ? *fold : edet_bngrad64{};
  if (k == 3) return fold ? dispatch_dwb_cpg<T, 3, true>(g, f, s) : dispatch_dwb_cpg<T, 3, false>(g, f, s);
  if (k == 5) return fold ? dispatch_dwb_cpg<T, 5, true>(g, f, s) : dispatch_dwb_cpg<T, 5, false>(g, f, s);
  set_error("dwconv_bwd: unsupported kernel %d", k);
  return EDET_EUNSUPPORTED;
}

// Kernel forms: TILE = k_dw_fwd / k_dw_wgrad / k_dw_dgrad (8x8 LDS tiles), DW3 = k_dw3
// (pipelined tiles), DIRECT = k_dw2_fwd / k_dw2_dgrad (one pixel per thread), DW4 =
// k_dw4_dgrad (register-blocked patches), ROWS = k_dws_fwd (row-streaming strips).  The
// per-shape choice below was measured with scripts/dw_probe.py / scripts/dw_sweep.py.
enum DwForm { DW_TILE = 0, DW_DW3 = 1, DW_DIRECT = 2, DW_DW4 = 3, DW_ROWS = 4 };

// block targets of the tile forms (kbench sweep 1024..8192: fwd 2048, wgrad 4096)
constexpr int DW_GRID_FWD = 2048, DW_GRID_WGRAD = 4096;

static DwForm dw_form_prod(int which, int K, int S, int C, int nseg);
static DwForm dw_form(int which, int K, int S, int C, int nseg, long rows_in) {
#ifdef EDET_DEV
  // development slot 27: force a form (1 TILE, 2 DW3, 3 DIRECT, 4 DW4, 5 ROWS) for route sweeps;
  // launch_dw falls back to a form the direction implements
  if (const int f = dev_knob(27)) return (DwForm)(f - 1);
#endif
  const bool direct_ok = C <= 2048;
  const bool dw4_ok = C % 8 == 0;  // channel rows split over blockIdx.y past 256 vectors
  if (which == 0) {
    // per-shape winners of scripts/dw_probe.py over the D0 b32 layers: the tile form with its
    // loads all in flight beats the direct form (which re-evaluates the lazy transform per
    // tap) everywhere; the pipelined tiles win where the double-buffered LDS still leaves
    // enough blocks per CU, and take C > 2048 (channel-blocked)
    // the row-streaming form (k_dws_fwd) wins every k5 shape (1.0-1.37x) and the k3 shapes
    // below; the 8x8 tiles keep k3 s2 at C = 96 (256^2 input: 194 vs 214 us) and k3 s1 at
    // C >= 480 (even, or 23 vs 29 us at 16^2 x 1152)
    // round-2 form sweep (kbench --dev): the 8x8 tiles for the C = 64 heads / BiFPN levels at
    // 32x32 and the pyramid (209 -> 192 us for the 8 head calls), rows for k3 s1 at
    // 32768 x 480 (63 -> 57 us)
    // round-3 form sweep (development slot 27, r03aa; the rows kernels lost their serial
    // filter-tap prologue this round): rows for the C = 64 pyramid (189 -> 174 us), k3 s2 at
    // C = 96 (166 -> 159) and k3 s1 at C >= 480 (16^2 x 1152: 24 -> 20); the 8x8 tiles keep the
    // single C = 64 BiFPN levels from 4096 to 32768 rows (43 vs 51 us at 32768)
    if (K == 3 && S == 1 && C == 64 && nseg == 1 && rows_in >= 4096 && rows_in <= 32768) return DW_TILE;
    if (K == 3 && S == 1 && C >= 480 && C <= 2048) return DW_ROWS;
    if (C <= 2048 && (K == 5 || (S == 1 && C <= 144) || (S == 2 && C >= 96))) return DW_ROWS;
    if ((K == 3 && S == 2 && C >= 192) || (S == 1 && C == 240) || C > 2048) return DW_DW3;
    return DW_TILE;
  }
  if (which == 1) {
    if (dw4_ok) return DW_DW4;
    return direct_ok ? DW_DIRECT : DW_TILE;
  }
  // wgrad: the row-streaming form wins 1.1-1.5x on single tensors up to C = 672 except k3 s2 at
  // C = 96 (256^2 input); the BiFPN / head pyramids (C = 64, five levels) keep the pipelined
  // tiles (30.4 vs 33.2 us), C = 1152 the 8x8 tiles (21.4 vs 25.6 us at k3)
  // round-2 sweep: the pipelined tiles for the small C = 64 BiFPN levels (8192 rows: 66 -> 48 us
  // over 6 calls), rows for the C = 64 pyramid (231 -> 223) and the k5 C = 1152 layers (96 -> 80)
  if (S == 1 && C == 64 && nseg == 1 && rows_in <= 8192) return DW_DW3;
  if (S == 1 && C == 64 && nseg > 1) return DW_ROWS;
  if (K == 5 && S == 1 && C == 1152) return DW_ROWS;
  // (k3 s2 at C = 240 took the rows form until round 3: 8x8 tiles 30 vs 32 us, r03aa)
  if (nseg == 1 && C <= 672 && (K == 5 || S == 1)) return DW_ROWS;
  return (S == 1 && (C <= 64 || (K == 5 && C == 240))) ? DW_DW3 : DW_TILE;
}

template <typename T, int K, int S>
static int launch_dw(int which, DwArgs g, hipStream_t s) {
  g.ncb = cdiv(g.C, DCB);
  long rows_in = 0;
  for (int i = 0; i < g.pin.nseg; ++i) rows_in += (long)g.pin.batch * g.pin.H[i] * g.pin.W[i];
  const DwForm form = dw_form(which, K, S, g.C, g.pin.nseg, rows_in);
  if (which == 0) {
    if (form == DW_ROWS) return dispatch_dws<T, K, S, false>(g, s);
    if (form == DW_DW3) return launch_dw3<T, K, S, false>(g, s);
    if (form == DW_TILE) {
      g.tiles_total = host_tiles(g.pout);
      const int G = std::max(1, std::min(g.tiles_total, cdiv(DW_GRID_FWD, g.ncb)));
      if (g.tiles_total) EDET_LAUNCH((k_dw_fwd<T, K, S>), dim3(G * g.ncb), dim3(256), 0, s, g);
      return check_launch("edet dwconv fwd");
    }
  } else if (which == 1) {
    if (form == DW_DW4) return launch_dw4_dgrad<T, K, S>(g, s);
    if (form == DW_TILE) {
      g.tiles_total = host_tiles(g.pin);
      if (g.tiles_total) EDET_LAUNCH((k_dw_dgrad<T, K, S>), dim3(g.tiles_total * g.ncb), dim3(256), 0, s, g);
      return check_launch("edet dwconv dgrad");
    }
  } else {
    if (form == DW_ROWS) return dispatch_dws<T, K, S, true>(g, s);
    if (form == DW_DW3) return launch_dw3<T, K, S, true>(g, s);
    g.tiles_total = host_tiles(g.pout);
    // ~4096 blocks: these loops are latency-bound (768 blocks measured 1.3-1.9x slower,
    // 4096 is 7 % faster than 2048)
    int chunks = cdiv(DW_GRID_WGRAD, g.ncb);
    if (chunks > g.tiles_total) chunks = g.tiles_total;
    if (chunks < 1) chunks = 1;
    g.tiles_per_wg = cdiv(g.tiles_total, chunks);
    chunks = cdiv(g.tiles_total, g.tiles_per_wg);
    g.part = nullptr;  // K*K*C is small: atomics measured faster than a 2048-way partial sum
    if (g.tiles_total) EDET_LAUNCH((k_dw_wgrad<T, K, S>), dim3(chunks * g.ncb), dim3(256), 0, s, g);
    return check_launch("edet dwconv wgrad");
  }
  // DW_DIRECT (fwd / dgrad)
  const DwGeom geo = dw_geom(g.C);
  const edet_pyramid& pp = which == 0 ? g.pout : g.pin;
  long px = 0;
  for (int i = 0; i < pp.nseg; ++i) px += (long)pp.batch * pp.H[i] * pp.W[i];
  const int grid = (int)std::max<long>(1, std::min<long>(4096, (px + geo.R - 1) / geo.R));
  if (which == 0) {
    const size_t lds = g.has_stats ? 2 * (size_t)geo.R * g.C * sizeof(float) : 0;
    if (px) EDET_LAUNCH((k_dw2_fwd<T, K, S>), dim3(grid), dim3(geo.TPR * geo.R), lds, s, g, geo);
  } else {
    if (px) EDET_LAUNCH((k_dw2_dgrad<T, K, S>), dim3(grid), dim3(geo.TPR * geo.R), 0, s, g, geo);
  }
  return check_launch("edet dwconv");
}

template <typename T>
static int dispatch_dw(int which, int k, int stride, const DwArgs& g, hipStream_t s) {
  if (k == 3 && stride == 1) return launch_dw<T, 3, 1>(which, g, s);
  if (k == 3 && stride == 2) return launch_dw<T, 3, 2>(which, g, s);
  if (k == 5 && stride == 1) return launch_dw<T, 5, 1>(which, g, s);
  if (k == 5 && stride == 2) return launch_dw<T, 5, 2>(which, g, s);
  set_error("dwconv: unsupported kernel %d stride %d", k, stride);
  return EDET_EUNSUPPORTED;
}

static int check_pyrs(const edet_pyramid* pin, const edet_pyramid* pout, int k, int stride) {
  EDET_REQUIRE(pin && pout && pin->nseg == pout->nseg && pin->batch == pout->batch &&
                   pin->nseg >= 1 && pin->nseg <= EDET_MAX_SEG,
               "dwconv: input/output pyramids disagree");
  for (int i = 0; i < pin->nseg; ++i)
    EDET_REQUIRE(pout->H[i] == cdiv(pin->H[i], stride) && pout->W[i] == cdiv(pin->W[i], stride),
                 "dwconv: segment %d output %dx%d != ceil(%dx%d / %d)", i, pout->H[i], pout->W[i],
                 pin->H[i], pin->W[i], stride);
  (void)k;
  return EDET_OK;
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_dwconv_fwd(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                    int stride, const void* w, void* y, const edet_pyramid* pout,
                    const edet_statout* stats, edet_stream_t stream) {
  EDET_REQUIRE(x && w && y, "dwconv_fwd: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0, "dwconv_fwd: need C%%8==0, ld%%8==0");
  int rc = check_pyrs(pin, pout, k, stride);
  if (rc) return rc;
  DwArgs g{};
  g.x = x->x; g.w = w; g.y = y; g.lz = *x; g.pin = *pin; g.pout = *pout; g.C = C;
  g.has_stats = stats != nullptr;
  if (stats) g.stats = *stats;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_dw<T>(0, k, stride, g, (hipStream_t)stream); });
}

int edet_dwconv_fwd_squeeze(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                            int stride, const void* w, void* y, const edet_pyramid* pout,
                            const edet_lazy* yv, double* s, edet_stream_t stream) {
  EDET_REQUIRE(x && w && y && yv && s, "dwconv_fwd_squeeze: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0, "dwconv_fwd_squeeze: need C%%8==0, ld%%8==0");
  EDET_REQUIRE(yv->gate == nullptr, "dwconv_fwd_squeeze: the squeezed value is the pre-gate one");
  EDET_REQUIRE(pin && pin->nseg == 1, "dwconv_fwd_squeeze: single tensors only (the SE is per image)");
  int rc = check_pyrs(pin, pout, k, stride);
  if (rc) return rc;
  if ((k != 3 && k != 5) || (stride != 1 && stride != 2)) {
    set_error("dwconv_fwd_squeeze: unsupported kernel %d stride %d", k, stride);
    return EDET_EUNSUPPORTED;
  }
  DwArgs g{};
  g.x = x->x; g.w = w; g.y = y; g.lz = *x; g.pin = *pin; g.pout = *pout; g.C = C;
  g.yv = *yv; g.sq = s; g.ncb = cdiv(C, DCB);
  // always the row-streaming form: the only one with the squeeze epilogue
  EDET_DTYPE_DISPATCH(dtype, T, {
    const hipStream_t st = (hipStream_t)stream;
    if (k == 3) return stride == 1 ? dispatch_dws<T, 3, 1, false>(g, st) : dispatch_dws<T, 3, 2, false>(g, st);
    return stride == 1 ? dispatch_dws<T, 5, 1, false>(g, st) : dispatch_dws<T, 5, 2, false>(g, st);
  });
}

int edet_dwconv_dgrad(int dtype, const void* dy, const edet_pyramid* pout, int C, int k,
                      int stride, const void* w, void* dx, const edet_pyramid* pin,
                      int accumulate, edet_stream_t stream) {
  EDET_REQUIRE(dy && w && dx, "dwconv_dgrad: null argument");
  EDET_REQUIRE(C % 8 == 0, "dwconv_dgrad: need C%%8==0");
  int rc = check_pyrs(pin, pout, k, stride);
  if (rc) return rc;
  DwArgs g{};
  g.dy = dy; g.w = w; g.dx = dx; g.pin = *pin; g.pout = *pout; g.C = C; g.accumulate = accumulate;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_dw<T>(1, k, stride, g, (hipStream_t)stream); });
}

int edet_dwconv_dgrad_fold(int dtype, const void* dy, const edet_pyramid* pout, int C, int k,
                           int stride, const void* w, void* dx, const edet_pyramid* pin,
                           const edet_lazy* xv, const edet_bngrad64* fold, edet_stream_t stream) {
  EDET_REQUIRE(dy && w && dx && xv && xv->x && fold, "dwconv_dgrad_fold: null argument");
  EDET_REQUIRE(C % 8 == 0 && xv->ld % 8 == 0, "dwconv_dgrad_fold: need C%%8==0, x->ld%%8==0");
  EDET_REQUIRE(xv->bn.enabled && xv->gate == nullptr, "dwconv_dgrad_fold: the folded value needs BN and no gate");
  int rc = check_pyrs(pin, pout, k, stride);
  if (rc) return rc;
  for (int i = 0; i < pin->nseg; ++i)
    EDET_REQUIRE(fold->dgamma[i] && fold->dbeta[i], "dwconv_dgrad_fold: null fold destination (segment %d)", i);
  // Route (kbench r04d, same box): the folded kernel wins the 256^2 k3 layer (2M x 96: 248 vs
  // 135 + 140 us for dgrad + reduce); at k5 and on smaller planes the patch kernel's extra x
  // stream costs more than the reduce pass it saves (524288 x 144 k5: 163 vs 57 + 52 us), so those
  // run the dgrad and then the reduce pass over (x, dx) -- same results, same destinations
  long rows_in = 0;
  for (int i = 0; i < pin->nseg; ++i) rows_in += (long)pin->batch * pin->H[i] * pin->W[i];
  if (!(k == 3 && rows_in >= (1L << 20))) {
    rc = edet_dwconv_dgrad(dtype, dy, pout, C, k, stride, w, dx, pin, 0, stream);
    if (rc) return rc;
    return edet_lazy_bwd_reduce(dtype, xv, pin, C, dx, nullptr, nullptr, fold, stream);
  }
  DwArgs g{};
  g.dy = dy; g.w = w; g.dx = dx; g.pin = *pin; g.pout = *pout; g.C = C; g.accumulate = 0;
  g.lz = *xv; g.x = xv->x;
  const hipStream_t st = (hipStream_t)stream;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (k == 3 && stride == 1) return launch_dw4_dgrad<T, 3, 1, true>(g, st, fold);
    if (k == 3 && stride == 2) return launch_dw4_dgrad<T, 3, 2, true>(g, st, fold);
    if (k == 5 && stride == 1) return launch_dw4_dgrad<T, 5, 1, true>(g, st, fold);
    if (k == 5 && stride == 2) return launch_dw4_dgrad<T, 5, 2, true>(g, st, fold);
    set_error("dwconv_dgrad_fold: unsupported kernel %d stride %d", k, stride);
    return EDET_EUNSUPPORTED;
  });
}

int edet_dwconv_wgrad(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                      int stride, const void* dy, const edet_pyramid* pout, float* dw,
                      edet_stream_t stream) {
  EDET_REQUIRE(x && dy && dw, "dwconv_wgrad: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0, "dwconv_wgrad: need C%%8==0 and ld%%8==0");
  int rc = check_pyrs(pin, pout, k, stride);
  if (rc) return rc;
  DwArgs g{};
  g.x = x->x; g.dy = dy; g.dw = dw; g.lz = *x; g.pin = *pin; g.pout = *pout; g.C = C;
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_dw<T>(2, k, stride, g, (hipStream_t)stream); });
}

int edet_dwconv_bwd(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                    int stride, const void* dy, const edet_pyramid* pout, const void* w,
                    void* dx, int accumulate, float* dw, const edet_bngrad64* fold,
                    edet_stream_t stream) {
  EDET_REQUIRE(x && dy && w && dx && dw, "dwconv_bwd: null argument");
  EDET_REQUIRE(C % 8 == 0 && x->ld % 8 == 0, "dwconv_bwd: need C%%8==0 and ld%%8==0");
  if (stride != 1) {
    set_error("dwconv_bwd: stride %d (the fused backward is stride 1; use edet_dwconv_dgrad/wgrad)", stride);
    return EDET_EUNSUPPORTED;
  }
  int rc = check_pyrs(pin, pout, k, stride);
  if (rc) return rc;
  EDET_REQUIRE(!fold || (!accumulate && x->gate == nullptr && x->bn.enabled),
               "dwconv_bwd: the BN fold needs accumulate == 0, no gate and a BatchNorm on x");
  DwArgs g{};
  g.x = x->x; g.lz = *x; g.dy = dy; g.w = w; g.dx = dx; g.dw = dw; g.pin = *pin; g.pout = *pout;
  g.C = C; g.accumulate = accumulate; g.ncb = cdiv(C, DCB);
  EDET_DTYPE_DISPATCH(dtype, T, { return dispatch_dwb<T>(k, g, fold, (hipStream_t)stream); });
}

int edet_dwconv_bwd_lazy(int dtype, const edet_lazy* x, const edet_pyramid* pin, int C, int k,
                         const edet_dgrad_lazy* dyl, const edet_pyramid* pout, const void* w,
                         void* dx, int accumulate, float* dw, const edet_bngrad64* fold,
                         edet_stream_t stream) {
  EDET_REQUIRE(x && dyl && dyl->dv && dyl->y.x && w && dx && dw, "dwconv_bwd_lazy: null argument");
  EDET_REQUIRE(C % DWT_CB == 0 && x->ld % 8 == 0 && dyl->y.ld == C,
               "dwconv_bwd_lazy: need C %% 16 == 0, x->ld %% 8 == 0 and y.ld == C");
  int rc = check_pyrs(pin, pout, k, 1);
  if (rc) return rc;
  EDET_REQUIRE(!fold || (!accumulate && x->gate == nullptr && x->bn.enabled),
               "dwconv_bwd_lazy: the BN fold needs accumulate == 0, no gate and a BatchNorm on x");
  if (dyl->y.bn.enabled)
    for (int i = 0; i < pout->nseg; ++i)
      EDET_REQUIRE(dyl->acc.dgamma[i] && dyl->acc.dbeta[i] && dyl->y.bn.sum[i] && dyl->y.bn.gamma[i],
                   "dwconv_bwd_lazy: null BN table of y (segment %d)", i);
  DwArgs g{};
  g.x = x->x; g.lz = *x; g.dyl = *dyl; g.w = w; g.dx = dx; g.dw = dw; g.pin = *pin; g.pout = *pout;
  g.C = C; g.accumulate = accumulate; g.ncb = cdiv(C, DCB);
  const edet_bngrad64 f = fold ? *fold : edet_bngrad64{};
  const hipStream_t st = (hipStream_t)stream;
  EDET_DTYPE_DISPATCH(dtype, T, {
    if (k == 3) return fold ? launch_dwt<T, 3, true, true>(g, f, st) : launch_dwt<T, 3, false, true>(g, f, st);
    if (k == 5) return fold ? launch_dwt<T, 5, true, true>(g, f, st) : launch_dwt<T, 5, false, true>(g, f, st);
    set_error("dwconv_bwd_lazy: unsupported kernel %d", k);
    return EDET_EUNSUPPORTED;
  });
}

}  // extern "C"
