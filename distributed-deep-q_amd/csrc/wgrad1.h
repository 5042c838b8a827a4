// conv1 weight gradient, direct form (gfx950).
//
// dW1[co][ky][kx][ci] = sum_{b,y,x} dconv1[b][y][x][co] * state[b][y+ky-3][x+kx-3][ci]
// db1[co]             = sum_{b,y,x} dconv1[b][y][x][co]
//
// conv1 has Cin = 4, so the implicit-GEMM form expands every input pixel 49x
// through global loads (15 VALU per MFMA measured).  Here one workgroup takes
// one image band of R rows: the input halo (R+6) x (W+6) x 4 is staged in LDS
// once and the band's dconv rows (W x 32 each) stream through two LDS slots,
// and 8 waves run MFMAs straight from LDS: wave ky (0..6) computes the 32 x 28 block
// (co) x (kx, ci) of tap row ky (lane n = kx*4 + ci; lanes 28..31 are padding
// whose products are dropped), wave 7 the bias column (B = 1).  K = the band's
// pixels, two per MFMA step.  Output: one fp32 slab per band in the layout
// of the wgrad slab reducer ([split][co][n], n = tap*4 + ci, bias at 196).
#pragma once
#include "common.h"

namespace ddq {

struct Wgrad1Args {
  int B, H, W, R;              // conv1 grid (H = W = S), band height
  int NP;                      // slab pitch (>= 197)
  const float* dconv;          // NHWC (B,H,W,32); droute: pooled (B,H/2,W/2,32)
  const uint8_t* droute;       // nullable: NHWC routing bytes of a pooled dconv (pool1's:
                               // 0..3 = routed quadrant dy*2+dx, 4 = ReLU'd window)
  const float* in;             // NHWC (B,H,W,4)  (the gathered state)
  float* part;                 // [B * H / R][32][NP]
};

// The band's dconv rows are streamed through two LDS row slots per half: row
// r+1 is loaded into registers before row r's MFMAs and stored after them,
// so only the first row's load is exposed (staging the whole band up front
// left every CU idle for the band's 64 KB load -- one workgroup per CU and a
// single wave of workgroups).  Sums run in the same order as before.
constexpr int kWgrad1Pre = 4;                // float4 of a dconv row per thread (W <= 256)

// Body of band `split` on 512 * NH threads with the dynamic LDS image `sm`.
template <int NH>
__device__ __forceinline__ void wgrad1_body(const Wgrad1Args& a, float* sm, int split) {
  const int W = a.W, R = a.R;
  const int PW = W + 6;
  const int RS = PW * 4 + 2;                 // odd-ish row stride: rows land on other banks
  float* patch = sm;                         // (R+6) x RS
  const int tid = threadIdx.x, lane = tid & 63, w = (tid >> 6) & 7, half = tid >> 9;
  const int ht = tid & 511;                  // thread within the half
  // this half's two dconv row slots, W x 32 each (16-B aligned)
  float* dslot = sm + (((R + 6) * RS + 3) & ~3) + half * 2 * W * 32;
  const int bands = a.H / R;
  const int b = split / bands, y0 = (split % bands) * R;
  const int rh = R / NH, rlo = half * rh;   // this half's rows of the band
  const int nd4 = W * 8;                    // float4 per dconv row
  const float4* drow = reinterpret_cast<const float4*>(a.dconv + ((size_t)b * a.H + y0) * W * 32);
  // named registers: a float4 array here was kept in scratch (80 B/lane)
  float4 p0 = f4zero(), p1 = f4zero(), p2 = f4zero(), p3 = f4zero();
  uint32_t m0 = 0, m1 = 0, m2 = 0, m3 = 0;
  static_assert(kWgrad1Pre == 4, "prefetch registers");
  // Pooled source (conv2's data gradient leaves the pool1-output gradient,
  // a quarter of the bytes): float4 f of full-res row y = pixel x = f/8,
  // channels 4*(f%8).. read pooled pixel (y/2, x/2) and its routing bytes,
  // and keep each channel only where the window routed quadrant (y&1, x&1).
  const uint8_t* __restrict__ route = a.droute;
  const int Wp = W >> 1;
  auto src_off = [&](int r, int f) -> size_t {
    return (((size_t)b * (a.H >> 1) + ((y0 + r) >> 1)) * Wp + ((f >> 3) >> 1)) * 32 + 4 * (f & 7);
  };
  auto load1 = [&](float4& p, uint32_t& m, int r, int f) {
    if (f >= nd4) return;
    if (!route) {
      p = drow[(size_t)r * nd4 + f];
    } else {
      const size_t o = src_off(r, f);
      p = *reinterpret_cast<const float4*>(a.dconv + o);
      m = *reinterpret_cast<const uint32_t*>(route + o);
    }
  };
  auto load_row = [&](int r) {
    load1(p0, m0, r, ht);
    load1(p1, m1, r, ht + 512);
    load1(p2, m2, r, ht + 1024);
    load1(p3, m3, r, ht + 1536);
  };
  auto store1 = [&](float4* d, float4 p, uint32_t m, int r, int f) {
    if (f >= nd4) return;
    if (route) {
      const uint32_t q = (((y0 + r) & 1) << 1) | ((f >> 3) & 1);
      p.x = (m & 0xff) == q ? p.x : 0.f;
      p.y = ((m >> 8) & 0xff) == q ? p.y : 0.f;
      p.z = ((m >> 16) & 0xff) == q ? p.z : 0.f;
      p.w = (m >> 24) == q ? p.w : 0.f;
    }
    d[f] = p;
  };
  auto store_row = [&](float* dst, int r) {
    float4* d = reinterpret_cast<float4*>(dst);
    store1(d, p0, m0, r, ht);
    store1(d, p1, m1, r, ht + 512);
    store1(d, p2, m2, r, ht + 1024);
    store1(d, p3, m3, r, ht + 1536);
  };
  load_row(rlo);

  // ---- stage the input halo (zero outside the image) ----
  for (int f = tid; f < (R + 6) * PW; f += 512 * NH) {
    const int py = f / PW, px = f % PW;
    const int gy = y0 - 3 + py, gx = px - 3;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)W)
      v = *reinterpret_cast<const float4*>(a.in + (((size_t)b * a.H + gy) * W + gx) * 4);
    float2* d = reinterpret_cast<float2*>(patch + py * RS + px * 4);
    d[0] = make_float2(v.x, v.y);
    d[1] = make_float2(v.z, v.w);
  }
  store_row(dslot, rlo);
  __syncthreads();

  const int l31 = lane & 31, h = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // A[co][k] = dconv[k][co]: lane (co = l31, half h) reads pixel 2s + h
  // B[k][n] = in[pixel + (ky, kx)][ci], n = kx*4 + ci = l31 (waves 0..6 = ky);
  // wave 7: the bias column (B = 1)
  const float* pb = patch + w * RS + 4 * h + l31;
  for (int i = 0; i < rh; ++i) {
    const int r = rlo + i;
    if (i + 1 < rh) load_row(r + 1);
    __builtin_amdgcn_sched_barrier(0);   // keep the next row's loads ahead of the MFMAs
    const float* ar = dslot + (i & 1) * W * 32 + h * 32 + l31;
    if (w < 7) {
      const float* br = pb + r * RS;
#pragma unroll 4
      for (int xs = 0; xs < W / 2; ++xs)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[xs * 64], br[xs * 8], acc, 0, 0, 0);
    } else {
#pragma unroll 4
      for (int xs = 0; xs < W / 2; ++xs)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[xs * 64], 1.0f, acc, 0, 0, 0);
    }
    // the other slot was last read in iteration i-1, fenced by its barrier
    if (i + 1 < rh) store_row(dslot + ((i + 1) & 1) * W * 32, r + 1);
    __syncthreads();
  }
  // ---- the two halves' partial sums meet in LDS (fixed order) ----
  if (NH == 2) {
    __syncthreads();
    float* red = sm;                                 // [8 waves][16][64]
    if (half == 1)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += red[(w * 16 + r) * 64 + lane];
  }
  // ---- epilogue: rows co = acc_row(r), column n = l31 ----
  float* slab = a.part + (size_t)split * 32 * a.NP;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (w < 7) {
      if (l31 < 28) slab[(size_t)co * a.NP + w * 28 + l31] = acc[r];
    } else if (l31 == 0) {
      slab[(size_t)co * a.NP + 196] = acc[r];
    }
  }
}

template <int NH>
__global__ __launch_bounds__(512 * NH) void wgrad1_kernel(const Wgrad1Args a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  wgrad1_body<NH>(a, sm, blockIdx.x);
}

inline size_t wgrad1_smem_bytes(int W, int R) {
  const int RS = (W + 6) * 4 + 2;
  const int NH = R == 8 ? 2 : 1;             // two row slots per half
  return (size_t)((((R + 6) * RS + 3) & ~3) + NH * 2 * W * 32) * 4;
}

// Band height: largest power of two <= 8 dividing H whose LDS image fits
// 96 KB (one workgroup per CU).  An 8-row band runs 16 waves (two halves of
// 4 rows summed in LDS): half the slabs of 4-row bands at the same waves.
inline int wgrad1_band(int H, int W) {
  int R = 8;
  while (R > 1 && (H % R != 0 || wgrad1_smem_bytes(W, R) > 96 * 1024)) R >>= 1;
  return R;
}

inline size_t wgrad1_launch_smem(const Wgrad1Args& a) {
  size_t shm = wgrad1_smem_bytes(a.W, a.R);
  if (a.R == 8 && shm < 8 * 16 * 64 * 4) shm = 8 * 16 * 64 * 4;   // halves' LDS sum
  return shm;
}

inline hipError_t launch_wgrad1(const Wgrad1Args& a, hipStream_t st) {
  if (a.W * 8 > 512 * kWgrad1Pre) return hipErrorInvalidValue;   // row prefetch registers
  const size_t shm = wgrad1_launch_smem(a);
  if (a.R == 8)
    hipLaunchKernelGGL(wgrad1_kernel<2>, dim3(a.B * (a.H / a.R)), dim3(1024), shm, st, a);
  else
    hipLaunchKernelGGL(wgrad1_kernel<1>, dim3(a.B * (a.H / a.R)), dim3(512), shm, st, a);
  return hipGetLastError();
}

}  // namespace ddq
