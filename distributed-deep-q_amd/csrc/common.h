// Shared device helpers for libddq_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#include <hip/hip_ext.h>

namespace ddq {

// Kernel timing (ddq_profile_step): when armed, the next launch through
// ddq_launch records these events at the dispatch's own start and end
// (hipExtLaunchKernel: the dispatch packet's timestamps, no marker packets
// around it), then disarms.  Thread-local: every ctx call runs on the
// caller's thread.
struct ExtTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local ExtTiming g_ext_timing;
// ddq_profile_step: while it enqueues a step, every launch no mark armed is
// counted (the step's table would silently miss its time)
extern thread_local bool g_profiling;
extern thread_local int g_unmarked;

template <class F, class... Args>
inline void ddq_launch(F kern, const dim3& grid, const dim3& block, uint32_t smem, hipStream_t s,
                       Args... args) {
  if (g_ext_timing.start) {
    const ExtTiming t = g_ext_timing;
    g_ext_timing = ExtTiming{};
    hipExtLaunchKernelGGL(kern, grid, block, smem, s, t.start, t.stop, 0, args...);
  } else {
    if (g_profiling) ++g_unmarked;
    hipLaunchKernelGGL(kern, grid, block, smem, s, args...);
  }
}

// Phase stamps of variant builds (make variant DEFS=-DDDQ_STAMPS, read by
// ddq_debug_stamps / tools/gpu/stamps.py): lane 0 of a workgroup records the
// 100 MHz real-time clock at a kernel's phase boundaries.  Empty otherwise.
#ifdef DDQ_STAMPS
constexpr int kStampSlots = 48, kStampBlocks = 512;
extern __device__ uint64_t g_stamps[kStampBlocks * kStampSlots];
#define DDQ_STAMP(slot)                                                        \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks)                         \
      g_stamps[blockIdx.x * kStampSlots + (slot)] = wall_clock64();            \
  } while (0)
#else
#define DDQ_STAMP(slot) do { } while (0)
#endif

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kActions = 4;        // barista/constants.py:8
constexpr int kFrames = 4;         // expgain.py:9
constexpr int kFc4 = 512;          // train_val.prototxt:169

// Division by a runtime constant (multiply-high + shift), exact for
// 0 <= n < 2^31 (Granlund-Montgomery / Hacker's Delight round-up method).
struct FastDiv {
  uint32_t d, mul, shr;
  FastDiv() = default;
  __host__ explicit FastDiv(uint32_t divisor) : d(divisor) {
    if (divisor == 1) { mul = 0; shr = 0; return; }
    uint32_t l = 0;
    while ((1ull << l) < divisor) ++l;
    uint64_t m = ((1ull << 32) * ((1ull << l) - divisor)) / divisor + 1;
    mul = (uint32_t)m;
    shr = l - 1;
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    if (d == 1) return n;
    uint32_t t = __umulhi(n, mul);
    return (t + ((n - t) >> 1)) >> shr;
  }
  __device__ __forceinline__ void divmod(uint32_t n, uint32_t& q, uint32_t& r) const {
    q = div(n);
    r = n - q * d;
  }
};

__device__ __forceinline__ float4 f4(float a, float b, float c, float d) {
  return make_float4(a, b, c, d);
}
__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// A kernel's dynamic-LDS limit is a per-device attribute: set it once per
// (kernel, device) -- `done` is the kernel's bitmask of devices already set
// (a race between threads only repeats the idempotent call).
inline hipError_t ensure_dyn_lds(const void* kern, std::atomic<uint64_t>& done, int bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? 1ull << dev : 0;
  if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.fetch_or(bit, std::memory_order_release);
  return e;
}

}  // namespace ddq
