// conv1 weight gradient, direct form (gfx950).
//
// dW1[co][ky][kx][ci] = sum_{b,y,x} dconv1[b][y][x][co] * state[b][y+ky-3][x+kx-3][ci]
// db1[co]             = sum_{b,y,x} dconv1[b][y][x][co]
//
// conv1 has Cin = 4, so the implicit-GEMM form expands every input pixel 49x
// through global loads (15 VALU per MFMA measured).  Here one workgroup takes
// one image band of R rows: the band's dconv rows (R x W x 32) and the input
// halo (R+6) x (W+6) x 4 are staged in LDS once, then 8 waves run MFMAs
// straight from LDS: wave ky (0..6) computes the 32 x 28 block
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
  const float* dconv;          // NHWC (B,H,W,32)
  const float* in;             // NHWC (B,H,W,4)  (the gathered state)
  float* part;                 // [B * H / R][32][NP]
};

template <int NH>
__global__ __launch_bounds__(512 * NH) void wgrad1_kernel(const Wgrad1Args a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int W = a.W, R = a.R;
  const int PW = W + 6;
  const int RS = PW * 4 + 2;                 // odd-ish row stride: rows land on other banks
  float* patch = sm;                         // (R+6) x RS
  float* dbuf = sm + (((R + 6) * RS + 3) & ~3);   // R*W x 32 (16-B aligned)
  const int tid = threadIdx.x, lane = tid & 63, w = (tid >> 6) & 7, half = tid >> 9;
  const int split = blockIdx.x;
  const int bands = a.H / R;
  const int b = split / bands, y0 = (split % bands) * R;

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
  // ---- stage the band's dconv rows (contiguous in NHWC) ----
  const float4* src = reinterpret_cast<const float4*>(a.dconv + ((size_t)b * a.H + y0) * W * 32);
  for (int f = tid; f < R * W * 8; f += 512 * NH)
    reinterpret_cast<float4*>(dbuf)[f] = src[f];
  __syncthreads();

  const int l31 = lane & 31, h = lane >> 5;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // A[co][k] = dconv[k][co]: lane (co = l31, half h) reads pixel 2s + h
  const float* pa = dbuf + h * 32 + l31;
  const int rh = R / NH, rlo = half * rh;           // this half's rows of the band
  if (w < 7) {
    // B[k][n] = in[pixel + (ky, kx)][ci], n = kx*4 + ci = l31
    const float* pb = patch + w * RS + 4 * h + l31;
    for (int r = rlo; r < rlo + rh; ++r) {
      const float* ar = pa + r * W * 32;
      const float* br = pb + r * RS;
#pragma unroll 4
      for (int xs = 0; xs < W / 2; ++xs)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[xs * 64], br[xs * 8], acc, 0, 0, 0);
    }
  } else {
    for (int r = rlo; r < rlo + rh; ++r) {
      const float* ar = pa + r * W * 32;
#pragma unroll 4
      for (int xs = 0; xs < W / 2; ++xs)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[xs * 64], 1.0f, acc, 0, 0, 0);
    }
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

inline size_t wgrad1_smem_bytes(int W, int R) {
  const int RS = (W + 6) * 4 + 2;
  return (size_t)((((R + 6) * RS + 3) & ~3) + R * W * 32) * 4;
}

// Band height: largest power of two <= 8 dividing H whose LDS image fits
// 96 KB (one workgroup per CU).  An 8-row band runs 16 waves (two halves of
// 4 rows summed in LDS): half the slabs of 4-row bands at the same waves.
inline int wgrad1_band(int H, int W) {
  int R = 8;
  while (R > 1 && (H % R != 0 || wgrad1_smem_bytes(W, R) > 96 * 1024)) R >>= 1;
  return R;
}

inline hipError_t launch_wgrad1(const Wgrad1Args& a, hipStream_t st) {
  size_t shm = wgrad1_smem_bytes(a.W, a.R);
  if (a.R == 8 && shm < 8 * 16 * 64 * 4) shm = 8 * 16 * 64 * 4;   // halves' LDS sum
  if (a.R == 8)
    hipLaunchKernelGGL(wgrad1_kernel<2>, dim3(a.B * (a.H / a.R)), dim3(1024), shm, st, a);
  else
    hipLaunchKernelGGL(wgrad1_kernel<1>, dim3(a.B * (a.H / a.R)), dim3(512), shm, st, a);
  return hipGetLastError();
}

}  // namespace ddq
