// fc4 forward / data-gradient kernels, register-direct MFMA (gfx950).
//
// fc4 is skinny (M = batch <= 32 per tile, N = 512, K = 64*(S/8)^2 = 4096 at
// 64x64): its cost is streaming W4 (8.4 MB per tower), not arithmetic.  The
// LDS-staged GEMM engine pays a global->LDS->MFMA round trip per K-step for
// operands that are used once, so these kernels feed v_mfma_f32_32x32x2_f32
// straight from registers: for a 32-deep k block, lane (l31, h) loads 16
// consecutive k of its row (four float4) and MFMA step j pairs k = 16h + j of
// both operands, so every wave issues all its weight loads up front (full
// memory-level parallelism); only the small activation tile goes through LDS.
#pragma once
#include "common.h"
#include "split.h"

namespace ddq {

__device__ __forceinline__ int fc_acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}
__device__ __forceinline__ float f4get(const float4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
// Bounds-checked buffer loads: an offset past `bytes` reads 0 with no branch
// or select, so every load of a wave can be issued before the first wait.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fc_rsrc(const float* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 fc_ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return *reinterpret_cast<float4*>(&v);
}
__device__ __forceinline__ float fc_ld1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
  return __builtin_bit_cast(float, v);
}
constexpr uint32_t kFcOOB = 0x80000000u;

// ---------------------------------------------------------------------------
// forward, split-K: part[split][z][b][n] = sum_{k in split} x[z][b][k] W4[z][n][k]
// grid (512/128, splits, nz), 4 waves; wave w owns n0 = 128*bx + 32*w, all b.
// x = pool3 in Caffe NCHW order (B, K); W4 Caffe (512, K).  K % 32 == 0.
// ---------------------------------------------------------------------------
constexpr int kFc4KLen = 128;                // k per split (64: head 6.6 -> 8.4 us; 256: fc4 fwd 6.0 -> 8.7)

struct Fc4FwdArgs {
  int B, K, nz;
  const float* x[2];
  const float* w[2];
  float* part;                     // [split][nz][B][512]
};

// The forward tile on the bf16 matrix cores with fp32-exact split operands
// (split.h; an f32-MFMA form's 64 cycles per 2 k left the wave's 64 MFMAs,
// 4096 cycles, behind its W4 loads).  Per 32-k block a lane's 16 consecutive
// k (16h .. 16h+15) are two 8-k halves, one per 32x32x16 step: step s pairs
// k = 16h + 8s + e of both operands (a permutation of the block's k, the
// same for A and B), 6 MFMAs a step (192 cycles against 1024 per block).  The
// x tile is split once while staged (3 bf16 planes in LDS, row stride
// 136 bf16: conflict-free b128 reads); the W values are split in registers.
__device__ __forceinline__ void split8(const float4& lo, const float4& hi, bf16x8& s0, bf16x8& s1,
                                       bf16x8& s2) {
  const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    __bf16 h, m, l;
    split3(v[e], h, m, l);
    s0[e] = h;
    s1[e] = m;
    s2[e] = l;
  }
}

// NWF waves per workgroup (32 n each: block bx covers n 32 NWF bx ..); the x
// tile in `smem` (3 planes of BT*32 rows of XSB bf16: fc4_fwd_smem_bytes)
template <int BT>
constexpr int fc4_fwd_smem_bytes() { return 3 * BT * 32 * (kFc4KLen + 8) * 2; }

template <int BT, int NWF = 4>
__device__ __forceinline__ void fc4_fwd_split_body(const Fc4FwdArgs& a, char* smem, int bx,
                                                   int by, int bzz) {
  constexpr int XSB = kFc4KLen + 8;     // bf16 per LDS row (272 B)
  constexpr int NT = 64 * NWF;
  __bf16 (*xs)[BT * 32 * XSB] = reinterpret_cast<__bf16 (*)[BT * 32 * XSB]>(smem);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int z = bzz % a.nz, split = by;
  const int bt0 = (bzz / a.nz) * (BT * 32);
  const int n0 = bx * (32 * NWF) + w * 32;
  const int K = a.K;
  const int k0 = split * kFc4KLen;
  const __amdgpu_buffer_rsrc_t rw = fc_rsrc(z ? a.w[1] : a.w[0], (uint32_t)(512 * K * 4));
  const __amdgpu_buffer_rsrc_t rx = fc_rsrc(z ? a.x[1] : a.x[0], (uint32_t)(a.B * K * 4));
  const uint32_t wrow = (uint32_t)((n0 + l31) * K + h * 16) * 4;

  f32x16 acc[BT], cor[BT];
#pragma unroll
  for (int t = 0; t < BT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[t][r] = 0.f; cor[t][r] = 0.f; }

  constexpr int kC4 = kFc4KLen / 4;
  constexpr int NX = BT * 32 * kC4 / NT;
  static_assert(NX * NT == BT * 32 * kC4, "x tile / workgroup");
  float4 xv[NX];
#pragma unroll
  for (int it = 0; it < NX; ++it) {
    const int f = threadIdx.x + NT * it;
    const int r = f / kC4, c4 = f % kC4;
    const int k = k0 + 4 * c4;
    xv[it] = fc_ld4(rx, k < K ? (uint32_t)((bt0 + r) * K + k) * 4 : kFcOOB);
  }
  float4 wv[kFc4KLen / 32][4];
#pragma unroll
  for (int kb = 0; kb < kFc4KLen / 32; ++kb) {
    const int k = k0 + kb * 32;
    const bool kin = k < K;
#pragma unroll
    for (int i = 0; i < 4; ++i) wv[kb][i] = fc_ld4(rw, kin ? wrow + (k + 4 * i) * 4 : kFcOOB);
  }
#pragma unroll
  for (int it = 0; it < NX; ++it) {
    const int f = threadIdx.x + NT * it;
    const int o = (f / kC4) * XSB + 4 * (f % kC4);
    const float v[4] = {xv[it].x, xv[it].y, xv[it].z, xv[it].w};
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 p0, p1, p2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      __bf16 hh, mm, ll;
      split3(v[e], hh, mm, ll);
      p0[e] = hh;
      p1[e] = mm;
      p2[e] = ll;
    }
    *reinterpret_cast<bf16x4*>(&xs[0][o]) = p0;
    *reinterpret_cast<bf16x4*>(&xs[1][o]) = p1;
    *reinterpret_cast<bf16x4*>(&xs[2][o]) = p2;
  }
  __syncthreads();
#pragma unroll
  for (int kb = 0; kb < kFc4KLen / 32; ++kb)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 b0, b1, b2;
      split8(wv[kb][2 * s], wv[kb][2 * s + 1], b0, b1, b2);
#pragma unroll
      for (int t = 0; t < BT; ++t) {
        const int o = (t * 32 + l31) * XSB + kb * 32 + 16 * h + 8 * s;
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(&xs[0][o]);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(&xs[1][o]);
        const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(&xs[2][o]);
        cor[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, cor[t], 0, 0, 0);
        cor[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, cor[t], 0, 0, 0);
        cor[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, cor[t], 0, 0, 0);
        cor[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, cor[t], 0, 0, 0);
        cor[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, cor[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[t], 0, 0, 0);
      }
    }
  const __amdgpu_buffer_rsrc_t rp = wt_rsrc(
      a.part, (uint32_t)((size_t)((a.K + kFc4KLen - 1) / kFc4KLen) * a.nz * a.B * 512 * 4));
  const uint32_t dbase = (uint32_t)((((size_t)(split * a.nz + z) * a.B) * 512 + n0 + l31) * 4);
#pragma unroll
  for (int t = 0; t < BT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int b = bt0 + t * 32 + fc_acc_row(r, lane);
      if (b < a.B) wt_store(rp, dbase + (uint32_t)b * 2048, acc[t][r] + cor[t][r]);
    }
}

template <int BT>
__global__ __launch_bounds__(256) void fc4_fwd_split_kernel(const Fc4FwdArgs a) {
  __shared__ __attribute__((aligned(16))) char xs[fc4_fwd_smem_bytes<BT>()];
  fc4_fwd_split_body<BT>(a, xs, blockIdx.x, blockIdx.y, blockIdx.z);
}

inline int fc4_fwd_splits(int K) { return (K + kFc4KLen - 1) / kFc4KLen; }

inline hipError_t launch_fc4_fwd(const Fc4FwdArgs& a, hipStream_t st) {
  if (a.B <= 32) {
    ddq_launch(fc4_fwd_split_kernel<1>, dim3(512 / 128, fc4_fwd_splits(a.K), a.nz),
                       dim3(256), 0, st, a);
  } else {
    const int nbt = (a.B + 63) / 64;
    ddq_launch(fc4_fwd_split_kernel<2>, dim3(512 / 128, fc4_fwd_splits(a.K), a.nz * nbt),
                       dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// data gradient fused with the pool3 un-pool:
// dx[b][kc] = sum_n dh4[b][n] W4[n][kc]  (kc Caffe order ch*S4^2 + p), then
// dconv3[b][2py+dy][2px+dx][ch] = (mask3[b][kc] == 2dy+dx) ? dx : 0.
// grid (K/32, ceil(B/32)); 8 waves split n (64 each) and are summed through
// LDS in fixed order.  A = dh4 rows (float4 along n), B = W4 columns (one
// dword per n, lanes along kc: coalesced 128-byte rows).
// ---------------------------------------------------------------------------
struct Fc4DgradArgs {
  int B, K, s4;
  FastDiv fS4sq, fS4;
  const float* dh4;                // (B, 512)
  const float* w4;                 // (512, K)
  const uint8_t* mask3;            // NCHW (B, 64, S4, S4); unused when pooled
  float* dconv3;                   // NHWC (B, 2S4, 2S4, 64), or pooled (B, S4, S4, 64)
  int pooled;                      // 1: write the pool3-output gradient only (NHWC);
                                   // its consumers expand it through pool3's routing
  __bf16* dsplit;                  // pooled: also split (split.h; conv3's weight
  int64_t dsplit_elems;            // gradient), plane stride dsplit_elems (nullable)
};

// Body on block (bx, by) with an 8 x 1024-float LDS image; 512 threads.
// SPLIT: the 32 f32 MFMAs of a wave (64 cycles each) as 24 bf16 ones on
// fp32-exact split operands (split.h; 32 cycles each): step s of a 32-n block
// pairs n = 16h + 8s + e of both operands, as fc4_fwd_split_kernel.
// KCW kc columns per block (32, or 16 -- the MFMA's other 16 columns read
// nothing and are dropped): K / 16 blocks fill the 256 CUs at 64x64, where
// K / 32 = 128 blocks streamed W4 on half of them (1.3 TB/s).
template <bool SPLIT, int KCW = 32>
__device__ __forceinline__ void fc4_dgrad_body(const Fc4DgradArgs& a, float (*red)[1024], int bx,
                                               int by) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int kc0 = bx * KCW, b0 = by * 32;
  const int K = a.K;
  const int nbase = w * 64 + h * 16;
  const __amdgpu_buffer_rsrc_t ra = fc_rsrc(a.dh4, (uint32_t)(a.B * 512 * 4));
  const __amdgpu_buffer_rsrc_t rb = fc_rsrc(a.w4, (uint32_t)(512 * K * 4));
  const uint32_t aoff = (uint32_t)((b0 + l31) * 512 + nbase) * 4;   // rows b >= B read 0
  const bool bcol = l31 < KCW;                                       // (wave-varying, no branch)
  const uint32_t boff = (uint32_t)(nbase * K + kc0 + l31) * 4;

  float4 av[2][4];
  float bv[2][16];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int j = 0; j < 16; ++j)
      bv[blk][j] = fc_ld1(rb, bcol ? boff + (uint32_t)((blk * 32 + j) * K) * 4 : kFcOOB);
#pragma unroll
  for (int blk = 0; blk < 2; ++blk)
#pragma unroll
    for (int i = 0; i < 4; ++i) av[blk][i] = fc_ld4(ra, aoff + (blk * 32 + 4 * i) * 4);
  __builtin_amdgcn_sched_barrier(0);   // keep every load ahead of the first MFMA
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  if (SPLIT) {
    f32x16 cor;
#pragma unroll
    for (int r = 0; r < 16; ++r) cor[r] = 0.f;
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a0, a1, a2, b0, b1, b2;
        split8(av[blk][2 * s], av[blk][2 * s + 1], a0, a1, a2);
        split8(make_float4(bv[blk][8 * s + 0], bv[blk][8 * s + 1], bv[blk][8 * s + 2],
                           bv[blk][8 * s + 3]),
               make_float4(bv[blk][8 * s + 4], bv[blk][8 * s + 5], bv[blk][8 * s + 6],
                           bv[blk][8 * s + 7]),
               b0, b1, b2);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, cor, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc, 0, 0, 0);
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += cor[r];
  } else {
#pragma unroll
    for (int blk = 0; blk < 2; ++blk)
#pragma unroll
      for (int j = 0; j < 16; ++j)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(av[blk][j >> 2], j & 3), bv[blk][j], acc,
                                                   0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][r * 64 + lane] = acc[r];
  __syncthreads();
  // 512 threads x 2 elements of the 32 x 32 tile; fixed-order wave sum
  const int H3 = 2 * a.s4;
#pragma unroll
  for (int e2 = 0; e2 < 2; ++e2) {
    const int e = threadIdx.x + 512 * e2;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) v += red[ww][e];
    const int r = e >> 6, ln = e & 63;
    const int bb = b0 + fc_acc_row(r, ln);
    const int kc = kc0 + (ln & 31);
    if (bb >= a.B || (ln & 31) >= KCW) continue;
    uint32_t ch, p, py, px;
    a.fS4sq.divmod((uint32_t)kc, ch, p);
    if (a.pooled) {   // one store per element instead of four (three of them zeros)
      const size_t o = ((size_t)bb * a.fS4sq.d + p) * 64 + ch;
      if (a.dconv3) a.dconv3[o] = v;
      if (a.dsplit) store_split(a.dsplit, a.dsplit_elems, o, v);
      continue;
    }
    a.fS4.divmod(p, py, px);
    const int mk = a.mask3[(size_t)bb * K + kc];
    float* base = a.dconv3 + (((size_t)bb * H3 + 2 * py) * H3 + 2 * px) * 64 + ch;
    base[0] = (mk == 0) ? v : 0.f;
    base[64] = (mk == 1) ? v : 0.f;
    base[(size_t)H3 * 64] = (mk == 2) ? v : 0.f;
    base[(size_t)H3 * 64 + 64] = (mk == 3) ? v : 0.f;
  }
}


}  // namespace ddq
