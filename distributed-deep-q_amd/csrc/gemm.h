// Generic fp32 MFMA GEMM engine for the deepq layers (gfx950).
//
//   C[m][n] = sum_k A(m,k) * B(k,n)      (exact f32 in / f32 accumulate)
//
// on v_mfma_f32_32x32x2_f32 (64 cycles / SIMD, 2048 MACs).  gfx950 has no
// xf32, so f32-input MFMA at the f32 vector rate (157.3 TF) is the matrix
// roofline for this fp32-parity workload.
//
// A problem type ``P`` supplies implicit operand loaders (im2col, unpooling,
// transposes are all folded into address arithmetic -- nothing is
// materialised) and an epilogue (bias + ReLU + 2x2 max-pool + argmax mask,
// un-pool scatter, split-K slab store ...):
//
//   static constexpr bool kAK4, kBK4;   // loader returns 4 consecutive k (true)
//                                       // or 4 consecutive m / n (false)
//   struct ACtx; struct BCtx;           // per-thread-slot state fixed over K
//   ACtx actx(int z, int m) const;      BCtx bctx(int z, int n) const;
//   struct KCtx; KCtx ktile(int z, int kb) const;   // per K-tile uniform state
//   float4 loadA(int z, const ACtx&, const KCtx&, int m, int k) const;
//   float4 loadB(int z, const BCtx&, const KCtx&, int k, int n) const;
//   void epilogue(int z, int split, int m0, int n0, const f32x16& acc, int lane) const;
//   int M, N, K, ksplit_len;            // K range per split (multiple of BK)
//
// Tiling: workgroup BM x BN, K-step BK, WM x WN x WK waves.  Each (wm, wn)
// wave group owns a (BM/WM) x (BN/WN) sub-tile of 32x32 MFMA blocks; the WK
// waves of a group split every K-step's depth between them (more waves per
// workgroup = more latency hiding and more MFMA work per barrier for the
// skinny / long-K shapes of this network) and are summed through LDS at the
// end.  Operands are staged global -> registers -> LDS with a two-buffer ring
// (one barrier per K-step; the next tile's global loads are in flight under
// the current tile's MFMAs).  LDS images are [k][m] / [k][n] so one wave-wide
// ds_read_b32 per operand and k-pair feeds an MFMA conflict-free (lanes 0-31
// and 32-63 read two 32-dword rows).
#pragma once
#include "common.h"

namespace ddq {

template <int BM_, int BN_, int BK_, int WM_, int WN_, int WK_ = 1>
struct GemmCfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_, WK = WK_;
  static constexpr int kThreads = 64 * WM * WN * WK;
  static constexpr int TM = BM / WM / 32;   // 32x32 blocks per wave along m
  static constexpr int TN = BN / WN / 32;
  static constexpr int APAD = 4, BPAD = 4;  // keeps float4 LDS writes aligned
  static constexpr int LDA = BM + APAD, LDB = BN + BPAD;
  static constexpr int KW = BK / WK;        // k depth per wave per K-step
  static constexpr int kStage = 2 * BK * (LDA + LDB);
  static constexpr int kRed = (WK - 1) * BM * BN;
  static constexpr int kSmem = kStage > kRed ? kStage : kRed;
  static_assert(TM >= 1 && TN >= 1, "wave tile must be >= 32x32");
  static_assert(BK % 4 == 0 && KW % 2 == 0 && BK % WK == 0, "bad BK / WK");
  static_assert(kSmem * 4 <= 160 * 1024, "LDS budget");
};

// Number of float4 slots each thread stages per K-step.
template <class C, int DIM>
struct Slots {
  static constexpr int kElems = DIM * C::BK / 4;
  static constexpr int kPer = (kElems + C::kThreads - 1) / C::kThreads;
};

// The GEMM body on block (bx, by = split, bz = tower) with an LDS image of
// C::kSmem floats; callable from fused launches (fc4_bwd_kernel) as well as
// from gemm_f32_kernel.  Threads >= C::kThreads must not enter.
template <class C, class P>
__device__ __forceinline__ void gemm_f32_body(const P& prob, float* smem, int bx, int by,
                                              int bz) {
  constexpr int BM = C::BM, BN = C::BN, BK = C::BK;
  constexpr int TM = C::TM, TN = C::TN;
  constexpr int LDA = C::LDA, LDB = C::LDB;
  using SA = Slots<C, BM>;
  using SB = Slots<C, BN>;

  float* As = smem;                    // [2][BK][LDA]
  float* Bs = smem + 2 * BK * LDA;     // [2][BK][LDB]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wk = wid / (C::WM * C::WN);
  const int w2 = wid % (C::WM * C::WN);
  const int wm = (w2 / C::WN) * (BM / C::WM);
  const int wn = (w2 % C::WN) * (BN / C::WN);

  const int z = bz;
  const int split = by;
  const int tiles_n = (prob.N + BN - 1) / BN;
  const int tm = bx / tiles_n;
  const int tn = bx % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = split * prob.ksplit_len;
  const int kend = min(prob.K, kbeg + prob.ksplit_len);
  const int nk = (kend - kbeg + BK - 1) / BK;

  // ---- per-slot loader contexts (fixed over the K loop) ----
  typename P::ACtx actx[SA::kPer];
  typename P::BCtx bctx[SB::kPer];
  int a_mn[SA::kPer], a_k[SA::kPer];
  int b_mn[SB::kPer], b_k[SB::kPer];
#pragma unroll
  for (int s = 0; s < SA::kPer; ++s) {
    int i = tid + s * C::kThreads;
    if (P::kAK4) { a_k[s] = (i % (BK / 4)) * 4; a_mn[s] = i / (BK / 4); }
    else         { a_mn[s] = (i % (BM / 4)) * 4; a_k[s] = i / (BM / 4); }
    actx[s] = prob.actx(z, m0 + a_mn[s]);
  }
#pragma unroll
  for (int s = 0; s < SB::kPer; ++s) {
    int i = tid + s * C::kThreads;
    if (P::kBK4) { b_k[s] = (i % (BK / 4)) * 4; b_mn[s] = i / (BK / 4); }
    else         { b_mn[s] = (i % (BN / 4)) * 4; b_k[s] = i / (BN / 4); }
    bctx[s] = prob.bctx(z, n0 + b_mn[s]);
  }

  float4 ra[SA::kPer], rb[SB::kPer];
  auto gload = [&](int kt) {
    const int kb = kbeg + kt * BK;
    const typename P::KCtx kc = prob.ktile(z, kb);   // K-tile-uniform decode (scalar)
#pragma unroll
    for (int s = 0; s < SA::kPer; ++s) {
      bool in = (SA::kElems % C::kThreads == 0) || (tid + s * C::kThreads) < SA::kElems;
      ra[s] = in ? prob.loadA(z, actx[s], kc, m0 + a_mn[s], kb + a_k[s]) : f4zero();
    }
#pragma unroll
    for (int s = 0; s < SB::kPer; ++s) {
      bool in = (SB::kElems % C::kThreads == 0) || (tid + s * C::kThreads) < SB::kElems;
      rb[s] = in ? prob.loadB(z, bctx[s], kc, kb + b_k[s], n0 + b_mn[s]) : f4zero();
    }
  };
  auto lstore = [&](int buf) {
    float* as = As + buf * BK * LDA;
    float* bs = Bs + buf * BK * LDB;
#pragma unroll
    for (int s = 0; s < SA::kPer; ++s) {
      if ((SA::kElems % C::kThreads) && (tid + s * C::kThreads) >= SA::kElems) continue;
      if (P::kAK4) {
        as[(a_k[s] + 0) * LDA + a_mn[s]] = ra[s].x;
        as[(a_k[s] + 1) * LDA + a_mn[s]] = ra[s].y;
        as[(a_k[s] + 2) * LDA + a_mn[s]] = ra[s].z;
        as[(a_k[s] + 3) * LDA + a_mn[s]] = ra[s].w;
      } else {
        *reinterpret_cast<float4*>(&as[a_k[s] * LDA + a_mn[s]]) = ra[s];
      }
    }
#pragma unroll
    for (int s = 0; s < SB::kPer; ++s) {
      if ((SB::kElems % C::kThreads) && (tid + s * C::kThreads) >= SB::kElems) continue;
      if (P::kBK4) {
        bs[(b_k[s] + 0) * LDB + b_mn[s]] = rb[s].x;
        bs[(b_k[s] + 1) * LDB + b_mn[s]] = rb[s].y;
        bs[(b_k[s] + 2) * LDB + b_mn[s]] = rb[s].z;
        bs[(b_k[s] + 3) * LDB + b_mn[s]] = rb[s].w;
      } else {
        *reinterpret_cast<float4*>(&bs[b_k[s] * LDB + b_mn[s]]) = rb[s];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int l31 = lane & 31;
  const int kh = lane >> 5;

  if (nk > 0) {
    gload(0);
    lstore(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const float* as = As + cur * BK * LDA + (wk * C::KW + kh) * LDA + wm + l31;
    const float* bs = Bs + cur * BK * LDB + (wk * C::KW + kh) * LDB + wn + l31;
#pragma unroll
    for (int kk = 0; kk < C::KW; kk += 2) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = as[kk * LDA + 32 * i];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = bs[kk * LDB + 32 * j];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  if constexpr (C::WK > 1) {
    // sum the WK partial accumulators of each (wm, wn) group through LDS
    float* red = smem;   // [(WK-1)][WM*WN][TM][TN][16][64]
    constexpr int per = TM * TN * 16 * 64;
    if (wk > 0) {
      float* dst = red + ((wk - 1) * C::WM * C::WN + w2) * per + lane;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((i * TN + j) * 16 + r) * 64] = acc[i][j][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int q = 1; q < C::WK; ++q) {
      const float* src = red + ((q - 1) * C::WM * C::WN + w2) * per + lane;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += src[((i * TN + j) * 16 + r) * 64];
    }
  }

  // Accumulator (i, j) register r of this lane holds
  //   row m = m0 + wm + 32 i + (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  //   col n = n0 + wn + 32 j + (lane & 31)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      prob.epilogue(z, split, m0 + wm + 32 * i, n0 + wn + 32 * j, acc[i][j], lane);
}

template <class C, class P>
__global__ __launch_bounds__(C::kThreads) void gemm_f32_kernel(const P prob) {
  __shared__ __attribute__((aligned(16))) float smem[C::kSmem];
  gemm_f32_body<C, P>(prob, smem, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Row of accumulator register r for a lane (see above).
__device__ __forceinline__ int acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

template <class C, class P>
inline hipError_t launch_gemm(const P& prob, int nz, int nsplit, hipStream_t st) {
  const int tiles = ((prob.M + C::BM - 1) / C::BM) * ((prob.N + C::BN - 1) / C::BN);
  dim3 grid(tiles, nsplit, nz);
  hipLaunchKernelGGL((gemm_f32_kernel<C, P>), grid, dim3(C::kThreads), 0, st, prob);
  return hipGetLastError();
}

}  // namespace ddq
