// Microbenchmark of the fc4 kernels in isolation (B = 32, K = 4096, two
// towers), with experimental variants.  Build: make -C tools/ubench
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../distributed-deep-q_amd/csrc/fc.h"

using namespace ddq;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// ---- variant: x tile staged once per workgroup in LDS ----
template <int KL>
__global__ __launch_bounds__(256) void fwd_ldsx(const Fc4FwdArgs a) {
  constexpr int XS = KL + 4;                 // padded row stride (floats)
  __shared__ __attribute__((aligned(16))) float xs[32 * XS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int z = blockIdx.z, split = blockIdx.y;
  const int n0 = blockIdx.x * 128 + w * 32;
  const int K = a.K, k0 = split * KL;
  const __amdgpu_buffer_rsrc_t rw = fc_rsrc(z ? a.w[1] : a.w[0], (uint32_t)(512 * K * 4));
  const float* x = z ? a.x[1] : a.x[0];
  const uint32_t wrow = (uint32_t)((n0 + l31) * K + h * 16) * 4;
  float4 wv[KL / 32][4];
#pragma unroll
  for (int kb = 0; kb < KL / 32; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) wv[kb][i] = fc_ld4(rw, wrow + (k0 + kb * 32 + 4 * i) * 4);
  // x tile: 32 rows x KL floats, float4 per thread-iteration
  constexpr int NX = 32 * KL / 4 / 256;
  float4 xv[NX];
#pragma unroll
  for (int it = 0; it < NX; ++it) {
    const int f = threadIdx.x + 256 * it;
    const int b = f / (KL / 4), c4 = f % (KL / 4);
    xv[it] = *reinterpret_cast<const float4*>(x + (size_t)b * K + k0 + 4 * c4);
  }
#pragma unroll
  for (int it = 0; it < NX; ++it) {
    const int f = threadIdx.x + 256 * it;
    const int b = f / (KL / 4), c4 = f % (KL / 4);
    *reinterpret_cast<float4*>(xs + b * XS + 4 * c4) = xv[it];
  }
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int kb = 0; kb < KL / 32; ++kb) {
    float4 xa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xa[i] = *reinterpret_cast<const float4*>(xs + l31 * XS + kb * 32 + h * 16 + 4 * i);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(xa[j >> 2], j & 3), f4get(wv[kb][j >> 2], j & 3),
                                                 acc, 0, 0, 0);
  }
  float* dst = a.part + ((size_t)(split * a.nz + z) * a.B) * 512 + n0 + l31;
#pragma unroll
  for (int r = 0; r < 16; ++r) dst[(size_t)fc_acc_row(r, lane) * 512] = acc[r];
}

// ---- variant: loads only (no MFMA): the memory phase of the current kernel ----
__global__ __launch_bounds__(256) void fwd_loadonly(const Fc4FwdArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int z = blockIdx.z, split = blockIdx.y;
  const int n0 = blockIdx.x * 128 + w * 32;
  const int K = a.K, k0 = split * kFc4KLen;
  const __amdgpu_buffer_rsrc_t rw = fc_rsrc(z ? a.w[1] : a.w[0], (uint32_t)(512 * K * 4));
  const __amdgpu_buffer_rsrc_t rx = fc_rsrc(z ? a.x[1] : a.x[0], (uint32_t)(a.B * K * 4));
  const uint32_t wrow = (uint32_t)((n0 + l31) * K + h * 16) * 4;
  float s = 0.f;
#pragma unroll
  for (int kb = 0; kb < kFc4KLen / 32; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 q = fc_ld4(rw, wrow + (k0 + kb * 32 + 4 * i) * 4);
      const float4 p = fc_ld4(rx, (uint32_t)(l31 * K + h * 16 + k0 + kb * 32 + 4 * i) * 4);
      s += q.x + q.y + q.z + q.w + p.x + p.y + p.z + p.w;
    }
  a.part[((size_t)(split * a.nz + z) * a.B) * 512 + n0 + lane] = s;
}

// ---- dgrad: loads only ----
__global__ __launch_bounds__(512) void dgrad_loadonly(const Fc4DgradArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int kc0 = blockIdx.x * 32;
  const int K = a.K;
  const int nbase = w * 64 + h * 16;
  const __amdgpu_buffer_rsrc_t rb = fc_rsrc(a.w4, (uint32_t)(512 * K * 4));
  const uint32_t boff = (uint32_t)(nbase * K + kc0 + l31) * 4;
  float s = 0.f;
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int j = 0; j < 16; ++j) s += fc_ld1(rb, boff + (uint32_t)((blk * 32 + j) * K) * 4);
  a.dconv3[blockIdx.x * 512 + threadIdx.x] = s;
}

// ---- dgrad variant: 16 waves per workgroup (n split 16 ways), 1024 threads ----
// and variant with kc blocks of 32 but workgroups split over n halves (2x WGs)
// writing partial dx to a buffer, summed by a second tiny pass (not the unpool)
template <int NW>
__global__ __launch_bounds__(64 * NW) void dgrad_nw(const Fc4DgradArgs a) {
  __shared__ float red[NW][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int kc0 = blockIdx.x * 32, b0 = 0;
  const int K = a.K;
  constexpr int NPW = 512 / NW;          // n per wave
  constexpr int NBLK = NPW / 32;
  const int nbase = w * NPW + h * 16;
  const __amdgpu_buffer_rsrc_t ra = fc_rsrc(a.dh4, (uint32_t)(a.B * 512 * 4));
  const __amdgpu_buffer_rsrc_t rb = fc_rsrc(a.w4, (uint32_t)(512 * K * 4));
  const uint32_t aoff = (uint32_t)((b0 + l31) * 512 + nbase) * 4;
  const uint32_t boff = (uint32_t)(nbase * K + kc0 + l31) * 4;
  float4 av[NBLK][4];
  float bv[NBLK][16];
#pragma unroll
  for (int blk = 0; blk < NBLK; ++blk) {
#pragma unroll
    for (int i = 0; i < 4; ++i) av[blk][i] = fc_ld4(ra, aoff + (blk * 32 + 4 * i) * 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) bv[blk][j] = fc_ld1(rb, boff + (uint32_t)((blk * 32 + j) * K) * 4);
  }
  __builtin_amdgcn_sched_barrier(0);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int blk = 0; blk < NBLK; ++blk)
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(av[blk][j >> 2], j & 3), bv[blk][j], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][r * 64 + lane] = acc[r];
  __syncthreads();
  for (int e = threadIdx.x; e < 1024; e += 64 * NW) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) v += red[ww][e];
    const int r = e >> 6, ln = e & 63;
    const int bb = fc_acc_row(r, ln);
    const int kc = kc0 + (ln & 31);
    a.dconv3[(size_t)bb * K + kc] = v;    // plain dx (no un-pool) for the timing study
  }
}

// ---- dgrad variant: VEC consecutive k per lane (float2 / float4 loads: 32*VEC*4-B
// contiguous runs per W4 row), VEC interleaved 32-column MFMA tiles (tile q:
// k = k0 + VEC*c + q), NW waves split n; fixed-order LDS reduction per tile ----
template <int VEC, int NW>
__global__ __launch_bounds__(64 * NW) void dgrad_vec(const Fc4DgradArgs a) {
  __shared__ float red[NW][1024];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int k0 = blockIdx.x * 32 * VEC;
  const int K = a.K;
  constexpr int NPW = 512 / NW;          // n per wave
  constexpr int NST = NPW / 2;           // MFMA steps (2 n each)
  const int nb = w * NPW + h * (NPW / 2);
  const __amdgpu_buffer_rsrc_t ra = fc_rsrc(a.dh4, (uint32_t)(a.B * 512 * 4));
  const __amdgpu_buffer_rsrc_t rb = fc_rsrc(a.w4, (uint32_t)(512 * K * 4));
  // A: dh4[b = l31][nb + j], j < NST (float4 chunks)
  float4 av[NST / 4];
#pragma unroll
  for (int i = 0; i < NST / 4; ++i) av[i] = fc_ld4(ra, (uint32_t)(l31 * 512 + nb + 4 * i) * 4);
  float bv[NST][VEC];
#pragma unroll
  for (int j = 0; j < NST; ++j) {
    const uint32_t off = (uint32_t)((nb + j) * K + k0 + VEC * l31) * 4;
    if (VEC == 4) {
      const float4 q = fc_ld4(rb, off);
      bv[j][0] = q.x; bv[j][1] = q.y; bv[j][2] = q.z; bv[j][VEC - 1] = q.w;
    } else {
      auto v = __builtin_amdgcn_raw_buffer_load_b64(rb, (int)off, 0, 0);
      bv[j][0] = __builtin_bit_cast(float, (uint32_t)v[0]);
      bv[j][1] = __builtin_bit_cast(float, (uint32_t)v[1]);
    }
  }
  f32x16 acc[VEC];
#pragma unroll
  for (int q = 0; q < VEC; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
#pragma unroll
  for (int j = 0; j < NST; ++j)
#pragma unroll
    for (int q = 0; q < VEC; ++q)
      acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(av[j >> 2], j & 3), bv[j][q], acc[q], 0, 0, 0);
#pragma unroll
  for (int q = 0; q < VEC; ++q) {
    if (q) __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) red[w][r * 64 + lane] = acc[q][r];
    __syncthreads();
    for (int e = threadIdx.x; e < 1024; e += 64 * NW) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) v += red[ww][e];
      const int r = e >> 6, ln = e & 63;
      const int bb = fc_acc_row(r, ln);
      const int kc = k0 + VEC * (ln & 31) + q;
      a.dconv3[(size_t)bb * K + kc] = v;
    }
  }
}

// ---- fwd variant: x tile loads issued before the W loads (the LDS barrier then
// waits for x only; the MFMAs of k block kb wait for its own W loads) ----
__global__ __launch_bounds__(256) void fwd_xfirst(const Fc4FwdArgs a) {
  constexpr int KL = kFc4KLen, XS = KL + 4;
  __shared__ __attribute__((aligned(16))) float xs[32 * XS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int z = blockIdx.z, split = blockIdx.y;
  const int n0 = blockIdx.x * 128 + w * 32;
  const int K = a.K, k0 = split * KL;
  const __amdgpu_buffer_rsrc_t rw = fc_rsrc(z ? a.w[1] : a.w[0], (uint32_t)(512 * K * 4));
  const __amdgpu_buffer_rsrc_t rx = fc_rsrc(z ? a.x[1] : a.x[0], (uint32_t)(a.B * K * 4));
  const uint32_t wrow = (uint32_t)((n0 + l31) * K + h * 16) * 4;
  constexpr int NX = 32 * KL / 4 / 256;
  float4 xv[NX];
#pragma unroll
  for (int it = 0; it < NX; ++it) {
    const int f = threadIdx.x + 256 * it;
    const int b = f / (KL / 4), c4 = f % (KL / 4);
    xv[it] = fc_ld4(rx, (uint32_t)(b * K + k0 + 4 * c4) * 4);
  }
  float4 wv[KL / 32][4];
#pragma unroll
  for (int kb = 0; kb < KL / 32; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) wv[kb][i] = fc_ld4(rw, wrow + (k0 + kb * 32 + 4 * i) * 4);
#pragma unroll
  for (int it = 0; it < NX; ++it) {
    const int f = threadIdx.x + 256 * it;
    const int b = f / (KL / 4), c4 = f % (KL / 4);
    *reinterpret_cast<float4*>(xs + b * XS + 4 * c4) = xv[it];
  }
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int kb = 0; kb < KL / 32; ++kb) {
    float4 xa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xa[i] = *reinterpret_cast<const float4*>(xs + l31 * XS + kb * 32 + h * 16 + 4 * i);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(xa[j >> 2], j & 3), f4get(wv[kb][j >> 2], j & 3),
                                                 acc, 0, 0, 0);
  }
  float* dst = a.part + ((size_t)(split * a.nz + z) * a.B) * 512 + n0 + l31;
#pragma unroll
  for (int r = 0; r < 16; ++r) dst[(size_t)fc_acc_row(r, lane) * 512] = acc[r];
}

template <class F>
float time_it(F f, int iters = 200) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) f();
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1000.f / iters;
}

int main() {
  const int B = 32, K = 4096, S4 = 8;
  float *x[2], *w[2], *part, *dh4, *dconv3, *dx;
  uint8_t* mask3;
  for (int z = 0; z < 2; ++z) {
    CK(hipMalloc(&x[z], B * K * 4));
    CK(hipMalloc(&w[z], 512 * K * 4));
    CK(hipMemset(x[z], 0, B * K * 4));
    CK(hipMemset(w[z], 0, 512 * K * 4));
  }
  CK(hipMalloc(&part, 64 * 2 * B * 512 * 4));
  CK(hipMalloc(&dh4, B * 512 * 4));
  CK(hipMalloc(&dconv3, B * K * 4 * 4));
  CK(hipMalloc(&dx, B * K * 4));
  CK(hipMalloc(&mask3, B * K));
  CK(hipMemset(dh4, 0, B * 512 * 4));
  CK(hipMemset(mask3, 0, B * K));
  // a large buffer to flush L2/MALL between launches when requested
  const size_t FL = (size_t)512 << 20;
  char* flush;
  CK(hipMalloc(&flush, FL));
  const bool doflush = getenv("FLUSH") != nullptr;
  auto fl = [&]() { if (doflush) CK(hipMemsetAsync(flush, 1, FL)); };

  Fc4FwdArgs fa;
  fa.B = B; fa.K = K; fa.nz = 2;
  fa.x[0] = x[0]; fa.x[1] = x[1]; fa.w[0] = w[0]; fa.w[1] = w[1]; fa.part = part;
  const int splits = fc4_fwd_splits(K);
  dim3 fg(4, splits, 2);
  auto r = [&](const char* name, float us, double bytes) {
    printf("%-28s %8.2f us  %7.2f TB/s(alg)\n", name, us, bytes / us / 1e6);
  };
  const double fbytes = 2.0 * 512 * K * 4 + 2.0 * B * K * 4 + 2.0 * splits * B * 512 * 4;
  float t_flush = doflush ? time_it([&] { fl(); }) : 0.f;
  auto T = [&](auto k) { return time_it([&] { fl(); k(); }) - t_flush; };
  r("fwd current", T([&] { hipLaunchKernelGGL(fc4_fwd_direct_kernel<1>, fg, dim3(256), 0, 0, fa); }), fbytes);
  r("fwd loads only", T([&] { hipLaunchKernelGGL(fwd_loadonly, fg, dim3(256), 0, 0, fa); }), fbytes);
  r("fwd x via LDS (KL128)", T([&] { hipLaunchKernelGGL(fwd_ldsx<128>, fg, dim3(256), 0, 0, fa); }), fbytes);
  {
    dim3 g2(4, K / 256, 2);
    const double b2 = 2.0 * 512 * K * 4 + 2.0 * B * K * 4 + 2.0 * (K / 256) * B * 512 * 4;
    r("fwd x via LDS (KL256)", T([&] { hipLaunchKernelGGL(fwd_ldsx<256>, g2, dim3(256), 0, 0, fa); }), b2);
    dim3 g3(4, K / 64, 2);
    const double b3 = 2.0 * 512 * K * 4 + 2.0 * B * K * 4 + 2.0 * (K / 64) * B * 512 * 4;
    r("fwd x via LDS (KL64)", T([&] { hipLaunchKernelGGL(fwd_ldsx<64>, g3, dim3(256), 0, 0, fa); }), b3);
  }

  Fc4DgradArgs da;
  da.B = B; da.K = K; da.s4 = S4; da.fS4sq = FastDiv(S4 * S4); da.fS4 = FastDiv(S4);
  da.dh4 = dh4; da.w4 = w[0]; da.mask3 = mask3; da.dconv3 = dconv3;
  const double dbytes = 512.0 * K * 4 + B * K * 4 * 4;
  da.pooled = 0; da.dsplit = nullptr; da.dsplit_elems = 0;
  r("dgrad unpooled (round 1)", T([&] { launch_fc4_dgrad_direct(da, 0); }), dbytes);
  {
    Fc4DgradArgs dp = da;
    dp.pooled = 1;
    r("dgrad pooled fp32 only", T([&] { launch_fc4_dgrad_direct(dp, 0); }), dbytes);
    __bf16* ds;
    CK(hipMalloc(&ds, 3 * B * K * 2));
    dp.dsplit = ds; dp.dsplit_elems = (int64_t)B * K;
    r("dgrad pooled fp32 + split (ship)", T([&] { launch_fc4_dgrad_direct(dp, 0); }), dbytes);
    dp.dconv3 = nullptr;
  }
  r("dgrad loads only", T([&] { hipLaunchKernelGGL(dgrad_loadonly, dim3(K / 32), dim3(512), 0, 0, da); }), dbytes);
  Fc4DgradArgs db = da;
  db.dconv3 = dx;
  r("dgrad 8 waves plain dx", T([&] { hipLaunchKernelGGL(dgrad_nw<8>, dim3(K / 32), dim3(512), 0, 0, db); }), dbytes);
  r("dgrad 16 waves plain dx", T([&] { hipLaunchKernelGGL(dgrad_nw<16>, dim3(K / 32), dim3(1024), 0, 0, db); }), dbytes);
  r("dgrad 4 waves plain dx", T([&] { hipLaunchKernelGGL(dgrad_nw<4>, dim3(K / 32), dim3(256), 0, 0, db); }), dbytes);
  r("dgrad vec2 8 waves", T([&] { hipLaunchKernelGGL((dgrad_vec<2, 8>), dim3(K / 64), dim3(512), 0, 0, db); }), dbytes);
  r("dgrad vec2 16 waves", T([&] { hipLaunchKernelGGL((dgrad_vec<2, 16>), dim3(K / 64), dim3(1024), 0, 0, db); }), dbytes);
  r("dgrad vec4 8 waves", T([&] { hipLaunchKernelGGL((dgrad_vec<4, 8>), dim3(K / 128), dim3(512), 0, 0, db); }), dbytes);
  r("dgrad vec4 16 waves", T([&] { hipLaunchKernelGGL((dgrad_vec<4, 16>), dim3(K / 128), dim3(1024), 0, 0, db); }), dbytes);
  r("fwd x loads first", T([&] { hipLaunchKernelGGL(fwd_xfirst, fg, dim3(256), 0, 0, fa); }), fbytes);
  r("empty-ish (memset 4B)", T([&] { CK(hipMemsetAsync(dx, 0, 4)); }), 4);
  CK(hipDeviceSynchronize());
  return 0;
}
