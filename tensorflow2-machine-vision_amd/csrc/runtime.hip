// Library-level entry points: error reporting, ABI version, async memset.
#include <limits.h>
#include <stdarg.h>
#include <stdio.h>
#include "common.hpp"

#include <algorithm>
#include <vector>

namespace edet {

static thread_local char g_err[512] = "";

// kernels launched by this thread since the last edet_launched_kernels() (base names)
static thread_local const char* g_launched[8];
static thread_local int g_nlaunched = 0;
void note_kernel(const char* site) {
  if (g_nlaunched < 8) g_launched[g_nlaunched] = site;
  if (g_nlaunched < INT_MAX) ++g_nlaunched;  // saturates when never queried (long eager runs)
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

#ifdef EDET_DEV
static int g_dev[64] = {};
int dev_knob(int slot) { return (slot >= 0 && slot < 64) ? g_dev[slot] : 0; }
#endif

// Caller-registered scratch for split reductions (weight gradients): blocks write partial
// results with plain stores, one reduce kernel sums them in a fixed order.  The library still
// allocates nothing; without a (large enough) workspace the kernels fall back to atomics.
static void* g_ws = nullptr;
static size_t g_ws_bytes = 0;

// Deferred split sums (ABI 10, edet_partials_defer / edet_partials_flush): inside a deferral
// window every split reduction takes a fresh region of the caller's deferral arena and its sum is
// recorded instead of launched; the flush sums every recorded job in one launch.  The weight
// gradients are read by nothing before the optimizer, and the D0 backward's 28 sum launches
// (~4.7 us each, mostly launch and drain) become one.  A region that does not fit falls back to
// the ordinary workspace and an immediate sum.
struct PartJob {
  const float* part;
  float* out;
  float* out2;
  long n, n2;
  int S, nblk;  // nblk: blocks of this job in the flush grid (x chunks)
  int atomic;   // another job adds into the same output: fp32 atomics
};
constexpr int PJ_MAX = 40;  // jobs per flush launch (kernel arguments)
static char* g_def = nullptr;
static size_t g_def_bytes = 0, g_def_used = 0, g_def_hw = 0;
static std::vector<PartJob> g_jobs;

float* workspace_f32(size_t n_floats) {
  if (g_def) {
    const size_t bytes = (n_floats * sizeof(float) + 255) & ~(size_t)255;
    if (g_def_used + bytes <= g_def_bytes) {
      float* p = (float*)(g_def + g_def_used);
      g_def_used += bytes;
      g_def_hw = std::max(g_def_hw, g_def_used);
      return p;
    }
    g_def_hw = std::max(g_def_hw, g_def_used + bytes);  // (reported: the arena the caller should give)
  }
  return (g_ws && n_floats * sizeof(float) <= g_ws_bytes) ? (float*)g_ws : nullptr;
}

// several zero fills in one launch (edet_zero_ranges): the step's per-step accumulators were
// one fill kernel each.  Chunk k of the concatenated ranges is 16 bytes of range i, first[i] <=
// k < first[i + 1]; a range's partial last chunk is written byte by byte
struct ZeroArgs {
  char* p[EDET_ZERO_MAX];
  long bytes[EDET_ZERO_MAX];
  long first[EDET_ZERO_MAX + 1];
  int n;
};
__global__ __launch_bounds__(256) void k_zero_ranges(ZeroArgs a) {
  const long total = a.first[a.n];
  for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < total; k += (long)gridDim.x * 256) {
    int i = 0;
    while (i + 1 < a.n && k >= a.first[i + 1]) ++i;
    const long off = (k - a.first[i]) * 16;
    if (off + 16 <= a.bytes[i]) {
      *reinterpret_cast<uint4*>(a.p[i] + off) = make_uint4(0u, 0u, 0u, 0u);
    } else {
      for (long b = off; b < a.bytes[i]; ++b) a.p[i][b] = 0;
    }
  }
}

// out[i] += sum_{s < S} part[s * n + i]: one thread per output and chunk of at most
// SUM_CHUNK partials (8 independent loads in flight).  A single chunk adds in a fixed order;
// more chunks (grid.y) spread the splits over the chip and add their sums with fp32 atomics
// (a few adders per address: a long dependent loop over hundreds of splits on the handful of
// blocks a small output needs was latency-bound)
constexpr int SUM_CHUNK = 32;
// Two outputs in one launch (a weight gradient's dW and db): the partials of the second,
// [S][n2], follow the first's [S][n] in the workspace; outputs i >= n map to out2[i - n].
__global__ __launch_bounds__(256) void k_sum_partials(const float* part, int S, long n, float* out, long n2,
                                                      float* out2) {
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n + n2) return;
  if (i >= n) {
    part += (size_t)S * n;
    i -= n;
    n = n2;
    out = out2;
  }
  const int s0 = blockIdx.y * SUM_CHUNK, s1 = min(S, s0 + SUM_CHUNK);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + 8 <= s1; s += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += part[(size_t)(s + u) * n + i];
  for (; s < s1; ++s) a[0] += part[(size_t)s * n + i];
  const float t = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  if (gridDim.y == 1) out[i] += t;
  else atomicAdd(out + i, t);
}

constexpr int SUM_CHUNK_DEF = SUM_CHUNK;
struct PartJobs {
  PartJob j[PJ_MAX];
  int n;
};
// the recorded sums, one launch: block b belongs to the job whose block range holds it (a scan
// over at most PJ_MAX kernel-argument entries), then k_sum_partials' loop
__global__ __launch_bounds__(256) void k_sum_partials_jobs(PartJobs a) {
  int b = blockIdx.x, j = 0;
  while (j < a.n - 1 && b >= a.j[j].nblk) b -= a.j[j++].nblk;
  const PartJob& J = a.j[j];
  const long nt = J.n + J.n2;
  const long bx = (nt + 255) / 256;
  const int chunk = (int)(b / bx);
  long i = (b - (long)chunk * bx) * 256 + threadIdx.x;
  if (i >= nt) return;
  const float* part = J.part;
  float* out = J.out;
  long n = J.n;
  if (i >= n) {
    part += (size_t)J.S * n;
    i -= n;
    n = J.n2;
    out = J.out2;
  }
  const int s0 = chunk * SUM_CHUNK_DEF, s1 = min(J.S, s0 + SUM_CHUNK_DEF);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + 8 <= s1; s += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += part[(size_t)(s + u) * n + i];
  for (; s < s1; ++s) acc[0] += part[(size_t)s * n + i];
  const float t = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (!J.atomic && J.nblk == bx) out[i] += t;
  else atomicAdd(out + i, t);
}

int sum_partials(const float* part, int S, long n, float* out, hipStream_t st, long n2, float* out2) {
  if (!out2) n2 = 0;
  if (n + n2 <= 0) return EDET_OK;
  if (g_def && (const char*)part >= g_def && (const char*)part < g_def + g_def_bytes) {
    PartJob j{};
    j.part = part; j.out = out; j.out2 = out2; j.n = n; j.n2 = n2; j.S = S;
    j.nblk = (int)(((n + n2 + 255) / 256) * ((S + SUM_CHUNK - 1) / SUM_CHUNK));
    g_jobs.push_back(j);
    return EDET_OK;
  }
  const unsigned chunks = (unsigned)((S + SUM_CHUNK - 1) / SUM_CHUNK);
  EDET_LAUNCH(k_sum_partials, dim3((unsigned)((n + n2 + 255) / 256), chunks), dim3(256), 0, st, part, S, n, out, n2,
              out2);
  return check_launch("edet sum_partials");
}

// Launch-duration probe: a single-thread kernel reading the constant-rate wall clock.  Placed
// before and after a launch on the same stream (also inside captured HIP graphs, where timing
// events are unavailable), it accumulates the launch's duration: slot = {t0, sum(t1-t0), n}.
__global__ void k_probe(unsigned long long* slot, int end) {
  const unsigned long long t = wall_clock64();
  if (!end) {
    slot[0] = t;
  } else {
    slot[1] += t - slot[0];
    slot[2] += 1;
  }
}

}  // namespace edet

extern "C" {

const char* edet_last_error(void) { return edet::g_err; }

int edet_abi_version(void) { return 10; }  // 3: edet_fuse_input.pool_arg; 4: opt norm partials; 5: dwconv_bwd; 6: dwconv_fwd_squeeze; 7: skip_nonfinite + opt_apply step; 8: bn_update_moving skip flag; 9: replicated statistics vectors; 10: one-pass fusion backward + fold

int edet_launched_kernels(char* buf, size_t size) {
  EDET_REQUIRE(buf && size > 0, "launched_kernels: null buffer");
  size_t o = 0;
  const int n = edet::g_nlaunched < 8 ? edet::g_nlaunched : 8;
  for (int i = 0; i < n; ++i) {
    const char* p = edet::g_launched[i];
    while (*p == '(' || *p == ' ') ++p;  // launch sites spell templates as (k_x<T, F>)
    if (i && o + 1 < size) buf[o++] = ',';
    for (; *p && *p != '<' && *p != ')' && o + 1 < size; ++p) buf[o++] = *p;
  }
  buf[o] = 0;
  const int total = edet::g_nlaunched;
  edet::g_nlaunched = 0;
  return total;
}

int edet_dev_set(int slot, int value) {
#ifdef EDET_DEV
  // a status like every entry point (returning the old value made a slot set to a
  // negative value read as "not a development build", and a bad slot number passed silently)
  EDET_REQUIRE(slot >= 0 && slot < 64, "edet_dev_set: slot %d outside 0..63", slot);
  edet::g_dev[slot] = value;
  return EDET_OK;
#else
  (void)slot;
  (void)value;
  edet::set_error("edet_dev_set: development slots exist only in the EDET_DEV build (make dev)");
  return EDET_EUNSUPPORTED;
#endif
}

int edet_partials_defer(void* arena, size_t bytes) {
  EDET_REQUIRE(arena && bytes > 0, "partials_defer: null arena");
  EDET_REQUIRE(!edet::g_def, "partials_defer: a deferral window is already open (edet_partials_flush first)");
  edet::g_def = (char*)arena;
  edet::g_def_bytes = bytes;
  edet::g_def_used = 0;
  edet::g_def_hw = 0;
  edet::g_jobs.clear();
  return EDET_OK;
}

int edet_partials_flush(size_t* needed, edet_stream_t stream) {
  EDET_REQUIRE(edet::g_def, "partials_flush: no deferral window open");
  using namespace edet;
  if (needed) *needed = g_def_hw;
  // outputs two jobs add into take atomics (the flush blocks of different jobs run concurrently)
  for (size_t a = 0; a < g_jobs.size(); ++a)
    for (size_t b = 0; b < g_jobs.size(); ++b)
      if (a != b && (g_jobs[a].out == g_jobs[b].out || (g_jobs[a].out2 && g_jobs[a].out2 == g_jobs[b].out2)))
        g_jobs[a].atomic = 1;
  int rc = EDET_OK;
  for (size_t j0 = 0; j0 < g_jobs.size() && rc == EDET_OK; j0 += PJ_MAX) {
    PartJobs a{};
    a.n = (int)std::min(g_jobs.size() - j0, (size_t)PJ_MAX);
    long nb = 0;
    for (int i = 0; i < a.n; ++i) {
      a.j[i] = g_jobs[j0 + i];
      nb += a.j[i].nblk;
    }
    EDET_LAUNCH(k_sum_partials_jobs, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, a);
    rc = check_launch("edet partials_flush");
  }
  g_jobs.clear();
  g_def = nullptr;
  g_def_bytes = g_def_used = 0;
  return rc;
}

int edet_set_workspace(void* ptr, size_t bytes) {
  edet::g_ws = ptr;
  edet::g_ws_bytes = ptr ? bytes : 0;
  return EDET_OK;
}

int edet_probe(uint64_t* slot, int end, edet_stream_t stream) {
  EDET_REQUIRE(slot, "probe: null slot");
  hipLaunchKernelGGL(edet::k_probe, dim3(1), dim3(1), 0, (hipStream_t)stream, (unsigned long long*)slot, end);
  return edet::check_launch("edet probe");
}

int edet_wall_clock_khz(int* khz) {
  EDET_REQUIRE(khz, "wall_clock_khz: null");
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess) {
    edet::set_error("wall clock rate: %s", hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

int edet_memset_async(void* p, int value, size_t bytes, edet_stream_t stream) {
  if (bytes == 0) return EDET_OK;
  EDET_REQUIRE(p != nullptr, "edet_memset_async: null pointer");
  hipError_t e = hipMemsetAsync(p, value, bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    edet::set_error("hipMemsetAsync: %s", hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

int edet_zero_ranges(int n, void* const* ptrs, const size_t* bytes, edet_stream_t stream) {
  EDET_REQUIRE(n >= 0 && n <= EDET_ZERO_MAX && (n == 0 || (ptrs && bytes)), "zero_ranges: 0..%d ranges", EDET_ZERO_MAX);
  edet::ZeroArgs a{};
  long chunks = 0;
  for (int i = 0; i < n; ++i) {
    EDET_REQUIRE(ptrs[i] != nullptr || bytes[i] == 0, "zero_ranges: null range %d", i);
    EDET_REQUIRE(((uintptr_t)ptrs[i] & 15) == 0, "zero_ranges: range %d not 16-byte aligned", i);
    a.p[a.n] = (char*)ptrs[i];
    a.bytes[a.n] = (long)bytes[i];
    a.first[a.n] = chunks;
    chunks += (long)((bytes[i] + 15) / 16);
    if (bytes[i]) ++a.n;
  }
  a.first[a.n] = chunks;
  if (chunks == 0) return EDET_OK;
  const int grid = (int)std::min<long>(1024, (chunks + 255) / 256);
  EDET_LAUNCH(edet::k_zero_ranges, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  return edet::check_launch("edet zero_ranges");
}

int edet_memcpy_async(void* dst, const void* src, size_t bytes, edet_stream_t stream) {
  if (bytes == 0) return EDET_OK;
  EDET_REQUIRE(dst && src, "edet_memcpy_async: null pointer");
  hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  if (e != hipSuccess) {
    edet::set_error("hipMemcpyAsync: %s", hipGetErrorString(e));
    return EDET_EHIP;
  }
  return EDET_OK;
}

}  // extern "C"
