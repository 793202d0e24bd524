// FETCH_SIZE / WRITE_SIZE calibration for the access patterns of the depthwise kernels
// (VERDICT r02 "calibrate the counters").  Each kernel moves a known number of bytes; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/bin/pmc_calib
//   rocprofv3 --pmc WRITE_SIZE --kernel-trace -- tools/bin/pmc_calib
// and compare the counter with the byte count printed here (MI355X_MICROARCH.md, HBM section:
// FETCH_SIZE reports half the bytes of 128-B coalesced reads; other widths uncalibrated).
//
// The tensor is [pixels][64] bf16 = 128 B per pixel (one line).  The depthwise kernels read
// 32 channels = 64 B per pixel (half a line) per block; which block reads the other half, and
// when, is the block-order question:
//   full        16-B lanes over whole lines (the guide's reference pattern)
//   half_outer  half h = block / nb outermost: the sibling half is read a whole pass later
//   half_inner  half h = block % 2: the sibling half is read by the neighbouring block id
//               (round-robin dispatch puts it on another XCD)
//   half_xcd    half h = block / 8 % 2: the sibling half on the same XCD (blocks b, b+8)
// Each is run at 64 MB (fits the 256 MB Infinity Cache) and 1 GB (does not), and timed with
// HIP events (median of 5) so the bandwidth cost of the pattern is measured beside the count.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

constexpr int PPB = 256;  // pixels per block (each thread: 16 B of 4 pixels' halves... see body)

// mode 0 full, 1 half_outer, 2 half_inner, 3 half_xcd.  Reads only; one dword per block out.
template <int MODE>
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ x, long npix, unsigned* out) {
  const int tid = threadIdx.x;
  uint32_t acc = 0;
  if constexpr (MODE == 0) {
    // block covers PPB/2 pixels x 128 B = 16 KB, 4 vectors per thread
    const long nvec = npix * 8;
    const long base = (long)blockIdx.x * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long v = base + u * 256 + tid;
      if (v < nvec) { const uint4 a = x[v]; acc ^= a.x ^ a.y ^ a.z ^ a.w; }
    }
  } else {
    // block covers PPB pixels x one 64-B half = 16 KB, 4 vectors per thread
    const long nb = (npix + PPB - 1) / PPB;
    long b = blockIdx.x, h;
    if (MODE == 1) { h = b / nb; b = b % nb; }
    else if (MODE == 2) { h = b & 1; b >>= 1; }
    else { h = (b >> 3) & 1; b = ((b >> 4) << 3) | (b & 7); }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * 256 + tid, p = e >> 2, q = e & 3;
      const long pix = b * PPB + p;
      if (pix < npix) { const uint4 a = x[pix * 8 + h * 4 + q]; acc ^= a.x ^ a.y ^ a.z ^ a.w; }
    }
  }
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // keeps the loads; practically never stores
}

// Writes of the same shapes: full lines, and 64-B halves with the sibling half outermost.
template <int MODE>
__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ y, long npix) {
  const int tid = threadIdx.x;
  const uint4 val = make_uint4(blockIdx.x, tid, 1, 2);
  if constexpr (MODE == 0) {
    const long nvec = npix * 8, base = (long)blockIdx.x * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long v = base + u * 256 + tid;
      if (v < nvec) y[v] = val;
    }
  } else {
    const long nb = (npix + PPB - 1) / PPB;
    long b = blockIdx.x, h;
    if (MODE == 1) { h = b / nb; b = b % nb; }
    else { h = b & 1; b >>= 1; }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * 256 + tid, p = e >> 2, q = e & 3;
      const long pix = b * PPB + p;
      if (pix < npix) y[pix * 8 + h * 4 + q] = val;
    }
  }
}

template <typename F>
static float time_ms(F f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> t;
  for (int i = 0; i < 5; ++i) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return t[2];
}

int main() {
  const long sizes[2] = {64L << 20, 1L << 30};
  const char* rnames[4] = {"full", "half_outer", "half_inner", "half_xcd"};
  const char* wnames[3] = {"wfull", "whalf_outer", "whalf_inner"};
  for (long bytes : sizes) {
    const long npix = bytes / 128;
    uint4* x;
    unsigned* out;
    CK(hipMalloc(&x, bytes));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMemset(x, 1, bytes));
    const unsigned g_full = (unsigned)((npix * 8 + 1023) / 1024);
    const unsigned g_half = (unsigned)(2 * ((npix + PPB - 1) / PPB));
    for (int m = 0; m < 4; ++m) {
      auto run = [&]() {
        if (m == 0) hipLaunchKernelGGL(k_read<0>, dim3(g_full), dim3(256), 0, 0, x, npix, out);
        if (m == 1) hipLaunchKernelGGL(k_read<1>, dim3(g_half), dim3(256), 0, 0, x, npix, out);
        if (m == 2) hipLaunchKernelGGL(k_read<2>, dim3(g_half), dim3(256), 0, 0, x, npix, out);
        if (m == 3) hipLaunchKernelGGL(k_read<3>, dim3(g_half), dim3(256), 0, 0, x, npix, out);
      };
      const float ms = time_ms(run);
      printf("read  %-12s bytes=%ld  %.3f ms  %.1f GB/s  (5 dispatches + this line's counter rows)\n", rnames[m],
             bytes, ms, bytes / ms / 1e6);
    }
    for (int m = 0; m < 3; ++m) {
      auto run = [&]() {
        if (m == 0) hipLaunchKernelGGL(k_write<0>, dim3(g_full), dim3(256), 0, 0, x, npix);
        if (m == 1) hipLaunchKernelGGL(k_write<1>, dim3(g_half), dim3(256), 0, 0, x, npix);
        if (m == 2) hipLaunchKernelGGL(k_write<2>, dim3(g_half), dim3(256), 0, 0, x, npix);
      };
      const float ms = time_ms(run);
      printf("write %-12s bytes=%ld  %.3f ms  %.1f GB/s\n", wnames[m], bytes, ms, bytes / ms / 1e6);
    }
    CK(hipDeviceSynchronize());
    CK(hipFree(x));
    CK(hipFree(out));
  }
  return 0;
}
