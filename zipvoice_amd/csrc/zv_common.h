// Shared device/host helpers for the ZipVoice MI355X (gfx950) engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>

// The 16-bit MFMA operand element.  `bf16` is bf16 in the default build; the fp16-operand
// build of the same sources (-DZV_OPERAND_F16, libzipvoice_hip_f16.so) makes it IEEE fp16:
// 11 significant bits instead of 8 at the same MFMA rate on gfx950 (v_mfma_f32_16x16x32_f16),
// the operand format of the parity-grade fast mode.  Every producer writes
// its GEMM operands through (bf16) casts (round to nearest even in either format).
#ifdef ZV_OPERAND_F16
typedef _Float16 bf16;
typedef _Float16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 bf16x2 __attribute__((ext_vector_type(2)));
#define ZV_MFMA_16x16x32 __builtin_amdgcn_mfma_f32_16x16x32_f16
#define ZV_MFMA_32x32x16 __builtin_amdgcn_mfma_f32_32x32x16_f16
#define ZV_OPERAND_NAME "fp16"
#else
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#define ZV_MFMA_16x16x32 __builtin_amdgcn_mfma_f32_16x16x32_bf16
#define ZV_MFMA_32x32x16 __builtin_amdgcn_mfma_f32_32x32x16_bf16
#define ZV_OPERAND_NAME "bf16"
#endif
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define ZV_CHECK(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +      \
                               " at " __FILE__ ":" + std::to_string(__LINE__) + ": " #expr); \
  } while (0)

// Host-blocking runtime calls (allocation and free, synchronous copies and memsets, device /
// stream / event synchronisation, stream / event / graph creation and destruction, copies to
// pageable host memory) are issued as ZV_BLOCKING(call): it counts them (zv_host_block_count in
// the C ABI) so a test can assert that a warm sample() issues none between its entry and its
// return (tests/test_gpu_host_sync.py); tests/test_host_block_scan.py checks on the CPU that no
// such call in csrc/ bypasses the counter.
#include <atomic>
static std::atomic<long long> g_zv_host_blocks{0};
#define ZV_BLOCKING(call) (g_zv_host_blocks.fetch_add(1, std::memory_order_relaxed), (call))

#define ZV_REQUIRE(cond, msg)                                                           \
  do {                                                                                  \
    if (!(cond)) throw std::invalid_argument(std::string(msg));                         \
  } while (0)

#define ZV_LAUNCH_CHECK() ZV_CHECK(hipGetLastError())

// ---------------------------------------------------------------------------
// numerics (scaling.py formulas, fp32)
// ---------------------------------------------------------------------------

// Transcendentals of the fused GEMM / conv epilogues are written on the hardware
// v_exp_f32 (2^x) / v_log_f32 (log2) / v_rcp_f32 forms (~1 ulp each): the libm
// forms (__expf/__logf/tanhf) cost 20-44 VALU per element, which at K = 512 is
// as long as the element's MFMA work.
__device__ __forceinline__ float fast_exp(float x) {
  return __builtin_amdgcn_exp2f(x * 1.44269504088896341f);
}
__device__ __forceinline__ float fast_ln(float x) {
  return __builtin_amdgcn_logf(x) * 0.693147180559945309f;
}

// SwooshLForward, scaling.py:1174-1180: log(1+exp(x-4)) (x-4 if inf) - 0.08x - 0.035, in
// base 2: t = log2(e) (x - 4); log(1 + e^(x-4)) = ln2 * max(log2(1 + 2^min(t, 126)), t) (the
// max is exact past t ~ 24 and takes over where 2^t would overflow).  6 VALU + 2 transcendental
// per element; every GEMM epilogue evaluates this one form, so a row's result does not depend
// on which kernel (tile size) a batch size selects
__device__ __forceinline__ float swoosh_l(float x) {
  const float t = fmaf(x, 1.44269504088896341f, -5.77078016355585362f);
  const float l = fmaxf(__builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(fminf(t, 126.0f))), t);
  return fmaf(l, 0.693147180559945309f, fmaf(x, -0.08f, -0.035f));
}
// SwooshRForward, scaling.py:1185-1191
__device__ __forceinline__ float swoosh_r(float x) {
  const float xo = x - 1.0f;
  float ls = fast_ln(1.0f + fast_exp(xo));
  ls = xo > 80.0f ? xo : ls;
  return ls - 0.08f * x - 0.313261687f;
}
// SwooshR module (SwooshRFunction without k2), scaling.py:1106-1116:
// logaddexp(0, x-1) - 0.08x - 0.313261687
__device__ __forceinline__ float swoosh_r_lae(float x) {
  float y = x - 1.0f;
  float m = fmaxf(y, 0.0f);
  return m + log1pf(expf(-fabsf(y))) - 0.08f * x - 0.313261687f;
}
// torch.sigmoid (GLU gate): 1 / (1 + e^-x)
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + fast_exp(-x));
}
// torch.tanh (NonlinAttention gate): 1 - 2 / (e^2x + 1); saturates to +-1 for |x| > 15
__device__ __forceinline__ float tanh_fast(float x) {
  const float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(fast_exp(2.0f * x) + 1.0f);
  return fabsf(x) > 15.0f ? copysignf(1.0f, x) : t;
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<bf16>(bf16 v) { return (float)v; }

template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float v) { return (bf16)v; }

// load 4 consecutive elements as floats (16-B for fp32, 8-B for bf16)
__device__ __forceinline__ void load4(const float* p, float (&v)[4]) {
  f32x4 t = *reinterpret_cast<const f32x4*>(p);
  v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
__device__ __forceinline__ void load4(const bf16* p, float (&v)[4]) {
  bf16x4 t = *reinterpret_cast<const bf16x4*>(p);
  v[0] = (float)t[0]; v[1] = (float)t[1]; v[2] = (float)t[2]; v[3] = (float)t[3];
}
__device__ __forceinline__ void store4(float* p, const float (&v)[4]) {
  f32x4 t = {v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p) = t;
}
__device__ __forceinline__ void store4(bf16* p, const float (&v)[4]) {
  bf16x4 t = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  *reinterpret_cast<bf16x4*>(p) = t;
}

__host__ __device__ static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
__host__ __device__ static inline long round_up(long a, long b) { return (a + b - 1) / b * b; }

// ---------------------------------------------------------------------------
// optional per-launch profiler (HIP events on the launch stream), used by
// bench.py to measure the dominant kernel's average duration live.
// ---------------------------------------------------------------------------
#include <vector>
#include <string>
struct ZvProfRec {
  std::string name;
  double flops;
  double bytes;
  hipEvent_t e0, e1;
};
struct ZvProfiler {
  bool on = false;
  bool detail = false;     // key GEMM records by shape (zv_profile(2))
  std::vector<ZvProfRec> recs;
};
extern ZvProfiler g_zv_prof;

struct ZvProfScope {
  ZvProfRec rec;
  hipStream_t s;
  bool active;
  ZvProfScope(const char* name, double flops, double bytes, hipStream_t st)
      : s(st), active(g_zv_prof.on) {
    if (active) {
      rec.name = name; rec.flops = flops; rec.bytes = bytes;
      (void)ZV_BLOCKING(hipEventCreate(&rec.e0));
      (void)ZV_BLOCKING(hipEventCreate(&rec.e1));
      (void)hipEventRecord(rec.e0, s);
    }
  }
  ~ZvProfScope() {
    if (active) {
      (void)hipEventRecord(rec.e1, s);
      g_zv_prof.recs.push_back(rec);
    }
  }
};

// compile-time loop: f(std::integral_constant<int, 0>) ... f(<N-1>)
template <class F, int... Is>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
