// Training-time image augmentation of the EfficientDet input pipeline on the GPU: the pixel
// half of datasets/coco_dataset_one.py:get_random_data (:99-126) -- box blur, perspective warp,
// additive noise -- followed by the proportional resize into the batch frame (:128) and the
// /255 normalisation (:134-135), all on device.  The box-corner geometry and the random draws
// stay on the host (augment.py), as in the reference.
//
// The reference runs these as OpenCV calls (cv2 is not in this image); each kernel restates the
// published OpenCV algorithm for 8-bit 3-channel images:
//   blur   cv2.blur(img, (k, k)) (image_helper.py:378-381): normalised box filter, anchor at
//          (k/2, k/2), BORDER_REFLECT_101, integer window sums, round half to even
//   warp   cv2.warpPerspective(img, M, (w, h), borderMode, borderValue) (image_helper.py:200-217):
//          inverse map in double per destination pixel (block-origin form of
//          WarpPerspectiveInvoker), source coordinates quantised to 1/32 pixel
//          (INTER_BITS = 5), bilinear taps with 15-bit fixed-point weights, BORDER_CONSTANT
//          (whole pixel = the border value when the 2x2 window misses the image, per tap
//          otherwise) or BORDER_REPLICATE (clamped taps)
//   noise  ImageHelper.opencvNoise (image_helper.py:245-257): + U{0..39} - 20 per element, clip
//          to [0, 255] (a counter-based hash keyed by (seed, element) instead of numpy's global
//          Mersenne Twister: same distribution, a different stream -- the drop-connect rule)
//   resize cv2.resize(INTER_AREA) into (rw, rh) + cv2.copyMakeBorder to the frame
//          (image_helper.py:293-322): area weights when shrinking, half-pixel bilinear when
//          enlarging, as data.resize_area restates them; the border constant or replicated
// Parity: the box geometry is bit-exact on the host; these pixel paths are parity-unpinned
// (no cv2 here) and property-tested (tests/test_augment_gpu.py).
#pragma clang fp contract(off)
#include <math.h>
#include "common.hpp"

namespace edet {

__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

// one thread per output pixel (3 channels)
__global__ void k_aug_blur(const uint8_t* src, int H, int W, int k, uint8_t* dst) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W, a = k / 2;
  int s0 = 0, s1 = 0, s2 = 0;
  for (int dy = 0; dy < k; ++dy) {
    const int yy = reflect101(y - a + dy, H);
    for (int dx = 0; dx < k; ++dx) {
      const uint8_t* p = src + ((size_t)yy * W + reflect101(x - a + dx, W)) * 3;
      s0 += p[0];
      s1 += p[1];
      s2 += p[2];
    }
  }
  const double inv = 1.0 / (double)(k * k);
  uint8_t* o = dst + (size_t)i * 3;
  o[0] = (uint8_t)min(255, (int)rint(s0 * inv));
  o[1] = (uint8_t)min(255, (int)rint(s1 * inv));
  o[2] = (uint8_t)min(255, (int)rint(s2 * inv));
}

__device__ __forceinline__ uint32_t mix32(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// dst (same size as src) = warp (+ noise).  m: the destination -> source map (row-major 3x3)
__global__ void k_aug_warp(const uint8_t* src, int H, int W, edet_aug_params p, uint8_t* dst) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= H * W) return;
  const int y = i / W, x = i - y * W;
  const double* M = p.warp;
  // WarpPerspectiveInvoker: the row terms at the 64-column block origin, then + M*x1
  const int xb = x & ~63, x1 = x - xb;
  const double X0 = M[0] * xb + M[1] * y + M[2];
  const double Y0 = M[3] * xb + M[4] * y + M[5];
  const double W0 = M[6] * xb + M[7] * y + M[8];
  double w = W0 + M[6] * x1;
  w = w != 0.0 ? 32.0 / w : 0.0;
  const double fX = fmax(-2147483648.0, fmin(2147483647.0, (X0 + M[0] * x1) * w));
  const double fY = fmax(-2147483648.0, fmin(2147483647.0, (Y0 + M[3] * x1) * w));
  const int X = (int)rint(fX), Y = (int)rint(fY);
  const int sx = max(-32768, min(32767, X >> 5)), sy = max(-32768, min(32767, Y >> 5));
  const int ax = X & 31, ay = Y & 31;
  // 15-bit fixed-point bilinear weights (exact for the 1/32 grid: they sum to 32768)
  const int w00 = (32 - ax) * (32 - ay) * 32, w01 = ax * (32 - ay) * 32;
  const int w10 = (32 - ax) * ay * 32, w11 = ax * ay * 32;
  int v[3];
  const bool inside = sx >= 0 && sx < W - 1 && sy >= 0 && sy < H - 1;
  if (p.warp_border == 0 && !inside && (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0)) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = p.warp_bg[c];
  } else {
    int x0 = sx, x1c = sx + 1, y0 = sy, y1 = sy + 1;
    bool ok00 = true, ok01 = true, ok10 = true, ok11 = true;
    if (!inside) {
      if (p.warp_border == 0) {
        const bool vx0 = x0 >= 0 && x0 < W, vx1 = x1c >= 0 && x1c < W;
        const bool vy0 = y0 >= 0 && y0 < H, vy1 = y1 >= 0 && y1 < H;
        ok00 = vx0 && vy0; ok01 = vx1 && vy0; ok10 = vx0 && vy1; ok11 = vx1 && vy1;
      }
      x0 = max(0, min(W - 1, x0)); x1c = max(0, min(W - 1, x1c));
      y0 = max(0, min(H - 1, y0)); y1 = max(0, min(H - 1, y1));
    }
    const uint8_t* p00 = src + ((size_t)y0 * W + x0) * 3;
    const uint8_t* p01 = src + ((size_t)y0 * W + x1c) * 3;
    const uint8_t* p10 = src + ((size_t)y1 * W + x0) * 3;
    const uint8_t* p11 = src + ((size_t)y1 * W + x1c) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int bg = p.warp_bg[c];
      const int s = (ok00 ? p00[c] : bg) * w00 + (ok01 ? p01[c] : bg) * w01 + (ok10 ? p10[c] : bg) * w10 +
                    (ok11 ? p11[c] : bg) * w11;
      v[c] = max(0, min(255, (s + (1 << 14)) >> 15));
    }
  }
  uint8_t* o = dst + (size_t)i * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    int t = v[c];
    if (p.noise) {
      const uint32_t h = mix32(p.noise_seed + 0x9E3779B97F4A7C15ull * (uint64_t)(3 * (size_t)i + c + 1));
      const float u = (float)(h >> 8) * (1.f / 16777216.f);  // [0, 1)
      t = max(0, min(255, t + (int)(u * 40.f) - 20));
    }
    o[c] = (uint8_t)t;
  }
}

// the resized image into the out_w x out_h frame, border filled, RGB /255 in the storage type
// (or raw uint8 with p.out_raw)
template <typename T>
__global__ void k_aug_resize(const uint8_t* src, int H, int W, edet_aug_params p, int oh, int ow, void* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= oh * ow) return;
  const int oy = i / ow, ox = i - oy * ow;
  int ry = oy - p.top, rx = ox - p.left;
  double v[3] = {0.0, 0.0, 0.0};
  const bool in = ry >= 0 && ry < p.rh && rx >= 0 && rx < p.rw;
  if (!in && p.pad_border == 0) {
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = p.pad_bg[c];
  } else {
    ry = max(0, min(p.rh - 1, ry));
    rx = max(0, min(p.rw - 1, rx));
    // separable weights of the output row / column (data.py _area_weights)
    double acc[3] = {0.0, 0.0, 0.0};
    auto axis = [](int d, int src_n, int dst_n, int& i0, int& i1, double& scale, double& a, double& b) {
      scale = (double)src_n / dst_n;
      if (dst_n <= src_n) {
        a = d * scale;
        b = (d + 1) * scale;
        i0 = (int)floor(a);
        i1 = min((int)ceil(b), src_n);
      } else {
        const double xx = (d + 0.5) * scale - 0.5;
        const int x0 = (int)floor(xx);
        a = xx - x0;  // fraction
        i0 = x0;
        i1 = x0 + 2;
      }
    };
    auto weight = [](int j, int src_n, int dst_n, double scale, double a, double b, int i0) {
      if (dst_n <= src_n) return (fmin(b, j + 1.0) - fmax(a, (double)j)) / scale;
      // enlarging: taps x0 (1 - t) and x0 + 1 (t), clamped to the image
      (void)b;
      const int c0 = min(max(i0, 0), src_n - 1), c1 = min(max(i0 + 1, 0), src_n - 1);
      return (j == c0 ? 1.0 - a : 0.0) + (j == c1 ? a : 0.0);
    };
    int y0, y1, x0, x1;
    double sy, ay, by, sx, ax, bx;
    axis(ry, H, p.rh, y0, y1, sy, ay, by);
    axis(rx, W, p.rw, x0, x1, sx, ax, bx);
    const int ylo = p.rh <= H ? y0 : max(0, y0), yhi = p.rh <= H ? y1 : min(H, y1);
    const int xlo = p.rw <= W ? x0 : max(0, x0), xhi = p.rw <= W ? x1 : min(W, x1);
    for (int xx = xlo; xx < xhi; ++xx) {
      const double wx = weight(xx, W, p.rw, sx, ax, bx, x0);
      if (wx == 0.0) continue;
      double col[3] = {0.0, 0.0, 0.0};
      for (int yy = ylo; yy < yhi; ++yy) {
        const double wy = weight(yy, H, p.rh, sy, ay, by, y0);
        const uint8_t* q = src + ((size_t)yy * W + xx) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) col[c] += wy * q[c];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += wx * col[c];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = fmin(255.0, fmax(0.0, rint(acc[c])));
  }
  if (p.out_raw) {
    uint8_t* o = (uint8_t*)out + (size_t)i * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = (uint8_t)v[c];
  } else {
    T* o = (T*)out + (size_t)i * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = from_f<T>((float)v[c] / 255.f);  // astype(float32) / 255
  }
}

}  // namespace edet

using namespace edet;

extern "C" {

int edet_augment_image(int dtype, const uint8_t* src, int H, int W, const edet_aug_params* p, uint8_t* scratch,
                       void* out, int out_h, int out_w, edet_stream_t stream) {
  EDET_REQUIRE(src && p && scratch && out, "augment_image: null argument");
  EDET_REQUIRE(H > 0 && W > 0 && out_h > 0 && out_w > 0 && (long)H * W < (1L << 30),
               "augment_image: bad sizes %dx%d -> %dx%d", H, W, out_h, out_w);
  EDET_REQUIRE(p->blur >= 0 && p->blur <= 31, "augment_image: blur size %d", p->blur);
  EDET_REQUIRE(p->rw >= 1 && p->rh >= 1 && p->top >= 0 && p->left >= 0 && p->top + p->rh <= out_h &&
                   p->left + p->rw <= out_w,
               "augment_image: resize box %dx%d at (%d, %d) outside the %dx%d frame", p->rw, p->rh, p->left, p->top,
               out_w, out_h);
  const hipStream_t s = (hipStream_t)stream;
  const unsigned nb = (unsigned)cdiv(H * W, 256);
  const uint8_t* cur = src;
  uint8_t* b0 = scratch;
  uint8_t* b1 = scratch + (size_t)H * W * 3;
  if (p->blur > 1) {
    EDET_LAUNCH(k_aug_blur, dim3(nb), dim3(256), 0, s, cur, H, W, p->blur, b0);
    cur = b0;
  }
  EDET_LAUNCH(k_aug_warp, dim3(nb), dim3(256), 0, s, cur, H, W, *p, cur == b0 ? b1 : b0);
  cur = cur == b0 ? b1 : b0;
  const unsigned no = (unsigned)cdiv(out_h * out_w, 256);
  EDET_DTYPE_DISPATCH(dtype, T, {
    EDET_LAUNCH(k_aug_resize<T>, dim3(no), dim3(256), 0, s, cur, H, W, *p, out_h, out_w, out);
    return check_launch("edet augment_image");
  });
}

}  // extern "C"
