// fp32-exact convolutions on the bf16 matrix cores (gfx950).
//
// gfx950 runs v_mfma_f32_32x32x16_bf16 at 16x the rate of the f32-input
// v_mfma_f32_32x32x2_f32 (2 vs 32 cycles per unit of K per SIMD).  An fp32
// value splits EXACTLY into three bf16 values, x = x0 + x1 + x2 (x0 = bf16(x),
// x1 = bf16(x - x0), x2 = bf16(x - x0 - x1): 3 x 8 significant bits = the 24
// of fp32; the remainder is below 2^-24 |x|).  A product of two split values
// is the sum of nine bf16 x bf16 products, each exact in fp32; the six with
// i + j <= 2 carry everything above 2^-24 |ab| (the three dropped ones are
// 2^-24, 2^-24 and 2^-32 of it, the size of fp32's own rounding), so
//
//   a . b  ~=  a0b0 + (a1b0 + a0b1 + a2b0 + a1b1 + a0b2)
//
// costs 6 bf16 MFMAs per 16 K instead of 8 f32 MFMAs at 4x the cycles:
// 192 against 512 cycles per 32x32x16 block, with fp32 accuracy (the big
// term and the five corrections accumulate in separate fp32 registers and
// are added once at the end).  The parity tests hold these kernels to the
// same per-element bound as the f32 MFMA path (tests/_parity.py).
//
// Storage: a "split tensor" of E elements is 3 bf16 planes of E (plane p at
// +p*E), each in the layout of the fp32 tensor it stands for.  Gradients are
// split once by their producer (the dgrad epilogue), weights by the apply /
// relayout; activations travel as fp32 (4 bytes a value instead of 6 through
// HBM) and are split while a consumer stages them into LDS.  Either way the
// MFMA loops only load: no conversion in any K loop.
//
// Direct convolution (fwd and dgrad), one workgroup = one image b x a TY x TX
// tile of output pixels x all N output channels, as in direct.h: the halo
// patch of all 3 planes is staged in LDS once, the weights tap by tap through
// a two-slot ring; lane (row r, k-half h) of the 32x32x16 operand reads the 8
// consecutive channels [16g + 8h, +8) of its pixel (A) or weight row (B) with
// one ds_read_b128 per plane.
#pragma once
#include <type_traits>

#include "common.h"

namespace ddq {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // native vector: promotable
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// x -> (x0, x1, x2) bf16, x0 + x1 + x2 == x to 2^-24 |x| (RNE conversions)
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r = x - (float)h;
  m = (__bf16)r;
  l = (__bf16)(r - (float)m);
}

// Write-through (sc1) vector store of one float at byte offset `off` of a
// buffer: the line is written to memory by the store itself, so the kernel's
// end leaves it clean (a kernel boundary otherwise writes back every dirty L2
// line the kernel left: ~B / 6 TB/s, MI355X_MICROARCH.md "boundary").
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void wt_store(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, (int)off, 0, 16);
}
__device__ __forceinline__ void wt_store4(__amdgpu_buffer_rsrc_t r, uint32_t off, float4 v) {
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, (int)off, 0, 16);
}
__device__ __forceinline__ void wt_store_b16(__amdgpu_buffer_rsrc_t r, uint32_t off, __bf16 v) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, v), r, (int)off, 0, 16);
}
__device__ __forceinline__ void wt_store_b8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint8_t v) {
  __builtin_amdgcn_raw_buffer_store_b8(v, r, (int)off, 0, 16);
}
// the split of v at element e of a split tensor of E elements, write-through
__device__ __forceinline__ void wt_store_split(__amdgpu_buffer_rsrc_t r, uint32_t E, uint32_t e,
                                               float v) {
  __bf16 h, m, l;
  split3(v, h, m, l);
  wt_store_b16(r, e * 2, h);
  wt_store_b16(r, (E + e) * 2, m);
  wt_store_b16(r, (2 * E + e) * 2, l);
}

// Keep-masks of 4 channels whose max-pool routing bytes (mw, values 0..4) name
// quadrant q (q4 = q * 0x01010101): 0xFFFF halves for the bf16 pairs (0,1)
// and (2,3).  Byte arithmetic instead of a compare + select per channel.
__device__ __forceinline__ void route_keep(uint32_t mw, uint32_t q4, uint32_t& k01,
                                           uint32_t& k23) {
  const uint32_t x = mw ^ q4;                                     // byte 0 iff routed to q
  const uint32_t nz = (x | (x >> 1) | (x >> 2)) & 0x01010101u;    // bytes <= 7: 1 iff not
  const uint32_t kb = (nz ^ 0x01010101u) * 0xFFu;                 // 0xFF iff routed to q
  k01 = __builtin_amdgcn_perm(kb, kb, 0x01010000u);
  k23 = __builtin_amdgcn_perm(kb, kb, 0x03030202u);
}

// The split planes of 8 consecutive fp32 values (a: values 0..3, b: 4..7) as
// three 16-byte vectors of bf16 pairs (v[p] = plane p; pair e = values 2e, 2e+1)
__device__ __forceinline__ void split_pack8(const float4& a, const float4& b, u32x4 (&v)[3]) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __bf16 h0, m0, l0, h1, m1, l1;
    split3(x[2 * e], h0, m0, l0);
    split3(x[2 * e + 1], h1, m1, l1);
    v[0][e] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    v[1][e] = (uint32_t)__builtin_bit_cast(uint16_t, m0) | ((uint32_t)__builtin_bit_cast(uint16_t, m1) << 16);
    v[2][e] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
  }
}

// Store the split of v at element e of a split tensor of E elements.
__device__ __forceinline__ void store_split(__bf16* t, int64_t E, int64_t e, float v) {
  __bf16 h, m, l;
  split3(v, h, m, l);
  t[e] = h;
  t[E + e] = m;
  t[2 * E + e] = l;
}

typedef short i16x4 __attribute__((ext_vector_type(4)));

// ds_read_b64_tr_b16 pair: lane 4q+p of a 16-lane group addresses row q,
// columns 4p..4p+3 of a 4-row block and receives column i of the four rows;
// two blocks (p0, p1) make one 8-element MFMA operand
__device__ __forceinline__ bf16x8 tr_pair(const __bf16* p0, const __bf16* p1) {
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  const i16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p0));
  const i16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p1));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  const i16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// bank-conflict-free strides for the 32x32x16 operand reads (tools/lds_banks.py):
// pixel stride CP + 8 bf16 (an odd number of 16-byte units), patch row stride
// == 128 (mod 256) bytes: the four 16-lane groups of a ds_read_b128 then hit
// 16 distinct 16-byte bank quads for TX = 16 tiles (two pixel rows per
// 32-pixel block); weight rows CP + 8 bf16 likewise.
// CPT input channels are processed in NCH = CPT / CP chunks of CP (the patch
// of one chunk is resident at a time: conv2 dgrad's 64-channel patch of a
// 16 x 16 tile would not fit LDS with its 3 planes).
// MF: the MFMA shape -- 0: v_mfma_f32_32x32x16_bf16 (32x32 blocks, k-steps of
// 16 channels), 1: v_mfma_f32_16x16x32_bf16 (a wave's 32x32 sub-tile as four
// 16x16 blocks, k-steps of 32 channels; the same operand bytes and MFMA
// cycles per FLOP).  MF = 1 reads lane l's 8 channels [8 (l / 16), +8) of row
// l % 16: pixel and weight-row strides CP + 16 bf16 (6 16-byte units) are
// conflict-free for it (a bank model of the four 16-lane groups).
template <int CPT, int CP, int N, int KS, int TY, int TX, int WM, int WN, int WK = 1, int MF = 0>
struct SplitCfg {
  static constexpr int NCH = CPT / CP;
  static constexpr int PH = TY + KS - 1, PW = TX + KS - 1;
  static constexpr int CS = CP + (MF ? 16 : 8);                       // bf16 per pixel
  static constexpr int RS0 = PW * CS;
  static constexpr int RS = RS0 + ((64 - (RS0 % 128)) + 128) % 128;   // == 64 (mod 128) bf16
  static constexpr int CW = CP + (MF ? 16 : 8);                       // bf16 per weight row
  static constexpr int T = KS * KS;
  static constexpr int KSTEP = CP / (MF ? 32 : 16);
  static constexpr int kGroup = 64 * WM * WN * WK;                     // all waves stage
  static constexpr int kThreads = kGroup;
  static constexpr int KSW = KSTEP / WK;                              // k-steps per wave
  // 32-row blocks per wave: the tile's NWIN pooling windows (8 per block),
  // padded to WM * TM * 8 -- padding rows read window 0 and are dropped by
  // the epilogue, so a tile need not hold a multiple of 32 pixels (10 x 20,
  // 10 x 10, ... tiles that fit the frame's edge: kernels.hip pick_tile)
  static constexpr int NWIN = TY * TX / 4;
  static constexpr int TM = (NWIN + 8 * WM - 1) / (8 * WM);
  static constexpr int TN = N / WN / 32;
  static constexpr int kPlane = PH * RS;                              // bf16 per patch plane
  static constexpr int kWSlot = N * CW;                               // bf16 per weight plane
  static constexpr int kPatchB = 3 * kPlane * 2;
  static constexpr int kWB = 2 * 3 * kWSlot * 2;                      // two-slot ring
  static constexpr int kSmemB = kPatchB + kWB;
  static_assert(CPT % CP == 0 && CP % 16 == 0 && TY % 2 == 0 && TX % 2 == 0, "shape");
  static_assert(TM >= 1 && TN >= 1 && (WM * TM - 1) * 8 < NWIN && N == WN * TN * 32, "wave tile");
  static_assert(kGroup <= 1024, "workgroup size");
  static_assert(kSmemB <= 160 * 1024, "LDS budget");
  static_assert(KSTEP % WK == 0, "k split");
  // every k group's accumulators for the fixed-order sums of the epilogue
  static_assert(WK == 1 || WK * WM * WN * 16 * 64 * 4 <= kSmemB, "k-split reduction");
  static_assert(4 % WK == 0, "epilogue windows per k group");
  static_assert(MF == 0 || CP % 32 == 0, "16x16x32: whole 32-channel k-steps");
};

// Row order of a 32-channel staging store (2 rows per 8-lane ds_write_b128
// group, SplitWStage::row): rows n and n + d share a group, d the row distance
// whose stride puts them 16 banks apart (d = 4 at 20 dwords, 2 at 24);
// identity for other shapes
template <int CP, int STRIDE>
__device__ __forceinline__ int pair_rows(int n0) {
  constexpr int DW = STRIDE / 2;                      // bf16 -> dwords
  constexpr int D = (CP == 32 && (4 * DW) % 32 == 16) ? 4 : (CP == 32 && (2 * DW) % 32 == 16) ? 2 : 0;
  if constexpr (D == 0) return n0;
  const int r = n0 & (2 * D - 1);
  return (n0 & ~(2 * D - 1)) | ((r >> 1) + (r & 1) * D);
}

// Weight staging of one (chunk, tap) (3 planes of N x CP bf16): a global ->
// register load issued two steps ahead, a register -> LDS store after the
// MFMAs of the step before it.  Native vector registers in an array indexed
// only by unrolled constants: HIP's uint4 struct (or registers captured by a
// lambda) were kept in scratch memory and every load waited on at once.
template <class C, int CPT, int CP, int N>
struct SplitWStage {
  static constexpr int WV = N * CP / 8;                         // 16-byte vectors per plane
  static constexpr int NVS = 3 * WV;                             // vectors per ring step
  static constexpr int kPer = (NVS + C::kGroup - 1) / C::kGroup;
  static_assert(kPer <= 12, "weight staging registers");
  u32x4 r[kPer];
  // ds_write_b128 serves 8 contiguous lanes per LDS cycle on banks (a/4) mod
  // 32.  With 32-channel rows (4 vectors) an 8-lane group writes two rows:
  // rows n and n + 1 overlap in 8 banks at a row stride of 20 dwords (CW 40)
  // or 24 (CW 48).  Rows n and n + d with d * stride = 16 (mod 32) take the
  // other 16 banks: conflict-free (a permutation of the rows within blocks of
  // 2d, the same for the load and the store of a lane)
  static __device__ __forceinline__ int row(int q) {
    return pair_rows<CP, C::CW>(q / (CP / 8));
  }

  // tap t of chunk ch
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t E, int ch, int t,
                                       int tid) {
#pragma unroll
    for (int S = 0; S < kPer; ++S) {   // clamped, unconditional: the store drops extra lanes
      const int f0 = tid + S * C::kGroup;
      const int f = NVS % C::kGroup == 0 || f0 < NVS ? f0 : NVS - 1;
      const int p = f / WV, q = f - p * WV;
      const int n = row(q), c8 = q % (CP / 8);
      r[S] = *reinterpret_cast<const u32x4*>(wk + p * E + ((size_t)n * C::T + t) * CPT + ch * CP +
                                             8 * c8);
    }
  }
  __device__ __forceinline__ void store(__bf16* dst, int tid) const {
#pragma unroll
    for (int S = 0; S < kPer; ++S) {
      const int f0 = tid + S * C::kGroup;
      // lanes past the vectors store nothing (whole waves at these sizes:
      // a uniform branch); they used to rewrite the last vector
      if (NVS % C::kGroup != 0 && f0 >= NVS) continue;
      const int f = NVS % C::kGroup == 0 || f0 < NVS ? f0 : NVS - 1;
      const int p = f / WV, q = f - p * WV;
      const int n = row(q), c8 = q % (CP / 8);
      *reinterpret_cast<u32x4*>(dst + p * C::kWSlot + n * C::CW + 8 * c8) = r[S];
    }
  }
};

struct SplitArgs {
  int B, H, W;               // conv grid (stride 1, same padding)
  int tiles_x;
  int pad;
  const __bf16* in[2];       // dgrad: split pooled NHWC (B,H/2,W/2,CPT)
  int64_t in_elems;          // E of the input split tensor
  const float* in32[2];      // fwd: the input activations, fp32 NHWC (B,H,W,CPT), split
                             // while staged
  const __bf16* wk[2];       // split weights [n][tap][CPT] (dgrad: transposed + flipped)
  int64_t wk_elems;          // E of the weight split tensor (plane stride)
  const float* bias[2];      // fwd
  float* out[2];             // fwd: fp32 pooled output (nullable), NHWC or NCHW (nchw)
  __bf16* out_split[2];      // fwd: split pooled NHWC output (nullable)
  int64_t out_elems;         // E of the pooled output
  int nchw;                  // fwd: fp32 output in Caffe (B,N,H/2,W/2) order
  uint8_t* mask[2];          // fwd: NHWC routing bytes (nullable)
  const uint8_t* in_route;   // dgrad: routing bytes of the pooled source (NHWC)
  const float* in_f32;       // dgrad: the pooled source in fp32 (B,H/2,W/2,CPT), split
                             // while staged (instead of in; conv3's, from fc4)
  float* pd;                 // dgrad: fp32 gradient of the previous pool output (nullable)
  __bf16* pd_split;          // dgrad: split gradient of the previous pool output (nullable)
  int64_t pd_elems;
  __bf16* xsplit;            // one channel chunk: the staged source split (dgrad: expanded),
  int64_t x_elems;           // NHWC (B,H,W,CPT), written once (nullable; fwd: tower 0 only)
                             // -- the layer's weight gradient reads it (wgrads)
  // conv2's data gradient only (N = 32): conv1's weight gradient fused in
  // (w1_tile_wgrad) -- w1_part non-null turns it on
  const uint8_t* w1_route;   // pool1's routing bytes, NHWC (B,H,W,32): the dgrad's grid
  const float* w1_in;        // conv1's input frames, fp32 NHWC (B,2H,2W,4)
  float* w1_part;            // slabs [B * tiles][32][w1_np], bias at column 196
  int w1_np;
};

// Epilogue of a direct conv tile (accumulator rows window-major: a lane's 4
// consecutive rows are one 2x2 pooling window).
//  fwd  : bias + ReLU + 2x2 max-pool + first-max routing byte; the pooled value
//         goes to the fp32 output (NHWC, or NCHW with nchw) and / or the split
//         NHWC output, the routing byte (0..3, 4 = ReLU'd window) to mask.
//  dgrad: the gradient of the previous layer's pool output, NHWC, fp32 and / or
//         split (the consumer routes it through that pool's mask).
// With WK k groups, group wkg finishes the windows gi (rows 4gi..4gi+3) with
// gi % WK == wkg.
template <int TM, int TN, int TX, int N, bool DGRAD, int WK = 1, int NWIN = 1 << 30>
__device__ __forceinline__ void split_epilogue(const SplitArgs& a, const f32x16 (&acc)[TM][TN],
                                               const float (&bpre)[TN], int b, int z, int y0,
                                               int x0, int wmi, int wni, int l31, int h,
                                               int wkg = 0) {
  float* __restrict__ outz = z ? a.out[1] : a.out[0];
  __bf16* __restrict__ osplit = z ? a.out_split[1] : a.out_split[0];
  uint8_t* __restrict__ maskz = z ? a.mask[1] : a.mask[0];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wni * TN * 32 + 32 * j + l31;
      if (!DGRAD) {
        const int Hp = a.H >> 1, Wp = a.W >> 1;
        const float bvv = bpre[j];   // loaded at the kernel's start
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (g % WK != wkg) continue;
          const int win = (mb + 8 * g + 4 * h) >> 2;
          if (win >= NWIN) continue;                // padding rows
          const int pyy = y0 / 2 + win / (TX / 2), pxx = x0 / 2 + win % (TX / 2);
          if (pyy >= Hp || pxx >= Wp) continue;
          const float v0 = acc[i][j][4 * g + 0] + bvv, v1 = acc[i][j][4 * g + 1] + bvv;
          const float v2 = acc[i][j][4 * g + 2] + bvv, v3 = acc[i][j][4 * g + 3] + bvv;
          float mx = v0; int arg = 0;
          if (v1 > mx) { mx = v1; arg = 1; }
          if (v2 > mx) { mx = v2; arg = 2; }
          if (v3 > mx) { mx = v3; arg = 3; }
          const bool pos = mx > 0.f;
          const float o = pos ? mx : 0.f;
          const size_t onhwc = (((size_t)b * Hp + pyy) * Wp + pxx) * N + n;
          // (plain stores: write-through measured no faster here, and slower
          // for the scattered NCHW pool3 and the routing bytes)
          if (outz) outz[a.nchw ? (((size_t)b * N + n) * Hp + pyy) * Wp + pxx : onhwc] = o;
          if (osplit) store_split(osplit, a.out_elems, onhwc, o);
          if (maskz) maskz[onhwc] = (uint8_t)(pos ? arg : 4);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if ((r >> 2) % WK != wkg) continue;
          const int m = mb + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int win = m >> 2;
          if (win >= NWIN) continue;                // padding rows
          const int y = y0 + 2 * (win / (TX / 2)) + ((m >> 1) & 1);
          const int x = x0 + 2 * (win % (TX / 2)) + (m & 1);
          if (y >= a.H || x >= a.W) continue;
          const size_t e = (((size_t)b * a.H + y) * a.W + x) * N + n;
          if (a.pd) a.pd[e] = acc[i][j][r];
          if (a.pd_split) store_split(a.pd_split, a.pd_elems, e, acc[i][j][r]);
        }
      }
    }
  }
}

// Forward epilogue through LDS: the pooled values of the tile (split planes
// or fp32, and the routing bytes) are first gathered in LDS in the output's
// own order, then copied out as whole 16-byte vectors (the accumulator layout
// gives 2-byte stores of 64-byte segments per plane and lane group and, for
// conv3's NCHW fp32 pool3, one 256-byte-strided dword per lane).  The stores
// of these one-round launches all leave at the end (A/B without them: conv1 /
// conv2 / conv3 forward -2.9 / -4.7 / -1.4 us); the 16-byte write-through form
// recovers ~1 us of it, the rest is the bytes themselves.  Every wave must have
// finished reading the patch / ring (the barrier at the top).  LDS: NWIN * N *
// 7 bytes.  One of out / out_split per launch (the forward passes never ask
// for both).
template <int TM, int TN, int TX, int N, int WK, int NWIN, int NT, int MF = 0>
__device__ __forceinline__ void split_epilogue_fwd_lds(const SplitArgs& a,
                                                       const f32x16 (&acc)[TM][TN],
                                                       const float (&bpre)[TN * (MF ? 2 : 1)],
                                                       char* smem, int b,
                                                       int z, int y0, int x0, int wmi, int wni,
                                                       int l31, int h, int wkg, int tid) {
  float* __restrict__ outz = z ? a.out[1] : a.out[0];
  __bf16* __restrict__ osplit = z ? a.out_split[1] : a.out_split[0];
  uint8_t* __restrict__ maskz = z ? a.mask[1] : a.mask[0];
  __bf16* sv = reinterpret_cast<__bf16*>(smem);                   // [3][NWIN][N] bf16 or
  float* fv = reinterpret_cast<float*>(smem);                     // [NWIN][N] fp32
  uint8_t* sm = reinterpret_cast<uint8_t*>(smem) + NWIN * N * 6;  // [NWIN][N]
  const bool split = osplit != nullptr;
  const int lane = l31 + 32 * h;
  if (!split && !a.nchw) {
    // fp32 NHWC (conv1 / conv2 forward: the next layer's input): straight
    // from the accumulators, no LDS gather and no barrier -- a store
    // instruction's lanes write whole 64-byte (16x16 blocks) or 128-byte
    // (32x32) runs of one pooled pixel's channels, its routing bytes likewise
    // (conv1 forward 10.6 -> 9.0 us, conv2 25.5 -> 25.2, same-box A/B)
    const int Hp = a.H >> 1, Wp = a.W >> 1;
    const __amdgpu_buffer_rsrc_t ro = wt_rsrc(outz, (uint32_t)(a.out_elems * 4));
    const __amdgpu_buffer_rsrc_t rm = wt_rsrc(maskz, maskz ? (uint32_t)a.out_elems : 0u);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (g % WK != wkg) continue;
          const int win = MF ? (mb + 16 * (g >> 1) + 4 * (lane >> 4)) >> 2 : (mb + 8 * g + 4 * h) >> 2;
          const int n = MF ? wni * TN * 32 + 32 * j + 16 * (g & 1) + (lane & 15)
                           : wni * TN * 32 + 32 * j + l31;
          const float bvv = MF ? bpre[2 * j + (g & 1)] : bpre[j];
          const int pyy = y0 / 2 + win / (TX / 2), pxx = x0 / 2 + win % (TX / 2);
          if (win >= NWIN || pyy >= Hp || pxx >= Wp) continue;   // padding rows / outside
          const float v0 = acc[i][j][4 * g + 0] + bvv, v1 = acc[i][j][4 * g + 1] + bvv;
          const float v2 = acc[i][j][4 * g + 2] + bvv, v3 = acc[i][j][4 * g + 3] + bvv;
          float mx = v0; int arg = 0;
          if (v1 > mx) { mx = v1; arg = 1; }
          if (v2 > mx) { mx = v2; arg = 2; }
          if (v3 > mx) { mx = v3; arg = 3; }
          const bool pos = mx > 0.f;
          const uint32_t e = (uint32_t)(((b * Hp + pyy) * Wp + pxx) * N + n);
          // write-through (plain stores of the same runs: no gain, A/B)
          wt_store(ro, e * 4, pos ? mx : 0.f);
          if (maskz) wt_store_b8(rm, e, (uint8_t)(pos ? arg : 4));
        }
      }
    }
    return;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (g % WK != wkg) continue;
        // element group g of the lane's accumulator: one pooling window x one
        // output channel (MF 0: 32x32 rows 8g + 4h + 0..3, column l31; MF 1:
        // 16x16 block (g >> 1, g & 1), rows 4 (lane >> 4) + 0..3, column lane & 15)
        const int win = MF ? (mb + 16 * (g >> 1) + 4 * (lane >> 4)) >> 2 : (mb + 8 * g + 4 * h) >> 2;
        const int n = MF ? wni * TN * 32 + 32 * j + 16 * (g & 1) + (lane & 15)
                         : wni * TN * 32 + 32 * j + l31;
        const float bvv = MF ? bpre[2 * j + (g & 1)] : bpre[j];
        if (win >= NWIN) continue;                // padding rows
        const float v0 = acc[i][j][4 * g + 0] + bvv, v1 = acc[i][j][4 * g + 1] + bvv;
        const float v2 = acc[i][j][4 * g + 2] + bvv, v3 = acc[i][j][4 * g + 3] + bvv;
        float mx = v0; int arg = 0;
        if (v1 > mx) { mx = v1; arg = 1; }
        if (v2 > mx) { mx = v2; arg = 2; }
        if (v3 > mx) { mx = v3; arg = 3; }
        const bool pos = mx > 0.f;
        const float o = pos ? mx : 0.f;
        const int e = win * N + n;
        if (split) {
          __bf16 hh, mm, ll;
          split3(o, hh, mm, ll);
          sv[e] = hh;
          sv[NWIN * N + e] = mm;
          sv[2 * NWIN * N + e] = ll;
        } else {
          fv[e] = o;
        }
        sm[e] = (uint8_t)(pos ? arg : 4);
      }
    }
  }
  __syncthreads();
  const int Hp = a.H >> 1, Wp = a.W >> 1;
  auto pix = [&](int win, int& off) {           // pooled NHWC pixel of window win
    const int pyy = y0 / 2 + win / (TX / 2), pxx = x0 / 2 + win % (TX / 2);
    off = (b * Hp + pyy) * Wp + pxx;
    return pyy < Hp && pxx < Wp;
  };
  // write-through (sc1) 16-byte stores: the lines go to memory as they are
  // written instead of at the kernel's end (conv1 / conv2 forward -0.9 / -0.5
  // us against plain stores of the same vectors)
  if (split) {
    constexpr int VPW = N / 8;                  // 16-byte vectors per window and plane
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const __amdgpu_buffer_rsrc_t rs = wt_rsrc(osplit + p * a.out_elems, (uint32_t)(a.out_elems * 2));
      for (int f = tid; f < NWIN * VPW; f += NT) {
        const int win = f / VPW, c = f % VPW;
        int off;
        if (!pix(win, off)) continue;
        __builtin_amdgcn_raw_buffer_store_b128(
            *reinterpret_cast<const u32x4*>(sv + (p * NWIN + win) * N + 8 * c), rs,
            (off * N + 8 * c) * 2, 0, 16);
      }
    }
  } else if (outz) {
    if (a.nchw) {   // Caffe (B, N, Hp, Wp): consecutive lanes walk a window row
      for (int f = tid; f < N * NWIN; f += NT) {
        const int n = f / NWIN, win = f % NWIN;
        const int pyy = y0 / 2 + win / (TX / 2), pxx = x0 / 2 + win % (TX / 2);
        if (pyy < Hp && pxx < Wp) outz[(((size_t)b * N + n) * Hp + pyy) * Wp + pxx] = fv[win * N + n];
      }
    } else {   // NHWC (the next layer's input: conv1 / conv2), write-through as above
      const __amdgpu_buffer_rsrc_t ro = wt_rsrc(outz, (uint32_t)(a.out_elems * 4));
      for (int f = tid; f < NWIN * (N / 4); f += NT) {
        const int win = f / (N / 4), c = f % (N / 4);
        int off;
        if (pix(win, off))
          wt_store4(ro, (uint32_t)((off * N + 4 * c) * 4), *reinterpret_cast<const float4*>(fv + win * N + 4 * c));
      }
    }
  }
  if (maskz) {
    constexpr int VPM = N / 16;                 // 16-byte vectors of routing bytes per window
    const __amdgpu_buffer_rsrc_t rm = wt_rsrc(maskz, (uint32_t)(a.B * Hp * Wp * N));
    for (int f = tid; f < NWIN * VPM; f += NT) {
      const int win = f / VPM, c = f % VPM;
      int off;
      if (!pix(win, off)) continue;
      __builtin_amdgcn_raw_buffer_store_b128(
          *reinterpret_cast<const u32x4*>(sm + win * N + 16 * c), rm, off * N + 16 * c, 0, 16);
    }
  }
}

// ---------------------------------------------------------------------------
// conv1's weight gradient fused into conv2's data gradient (backward of
// train_val.prototxt:39-61; conv1 has no bottom diff).  A data-gradient tile
// ends with dpool1 at its TY x TX pool1 pixels; through pool1's routing bytes
// that is dconv1 at the 2TY x 2TX conv1 pixels under them, and those pixels'
// share of
//   dW1[co][ky][kx][ci] = sum_p dconv1[p][co] frame[p + (ky-3, kx-3)][ci]
//   db1[co]             = sum_p dconv1[p][co]
// needs nothing else but the frames' halo.  So the workgroup scatters its
// dpool1 values (split, split.h split3) into an LDS image of the expanded
// dconv1 rows, stages the halo (frames are integers: exact in bf16, ONE
// plane), runs conv1's MFMAs over its own pixels and writes its fp32 slab for
// the slab reduce (fixed order: deterministic, no atomics).  dpool1 never
// leaves the workgroup: round 3 wrote it split (6.3 MB at 64x64 B = 32) for a
// separate 14 us launch that re-read and re-expanded it.
//
// MFMA form (as round 3's standalone kernel): A = dconv1 (32 co x 16 pixels of
// a row), B = frames (16 pixels x n = 4 kx + ci, kx 0..7: column 28..31 is a
// zero tap, dropped), both read with ds_read_b64_tr_b16 out of pixel-major
// rows; the halo row is stored with pixel stride 4 bf16, so tap row ky's B is
// one transposed read of halo row y + ky at offset 4x + n.  Work unit = (tap
// row ky, 16-pixel column segment): 3 MFMAs (the three dconv1 planes x the
// exact frame) per conv1 row of the tile; a unit's sums over the segments
// meet in LDS in fixed order.
// ---------------------------------------------------------------------------
template <int TY, int TX, int NT>
struct W1Fuse {
  static constexpr int R = 2 * TY;                  // conv1 rows of the tile
  static constexpr int XW = (2 * TX + 15) & ~15;    // conv1 pixels per row, whole k-steps
  static constexpr int NSEG = XW / 16;
  static constexpr int PSD = 32;                    // bf16 per pixel (32 channels, 64 B:
                                                    // conflict-free transposed reads)
  static constexpr int XPL = R * XW * PSD;          // bf16 per dconv1 plane
  static constexpr int HR = R + 6;                  // halo rows
  static constexpr int HW = XW + 6;                 // halo pixels per row
  static constexpr int IROW = 4 * HW + 64;          // bf16 per halo row (+ the read tail)
  static constexpr int kXB = 3 * XPL * 2;
  static constexpr int kHaloB = HR * IROW * 2;
  static constexpr int NU = 7 * NSEG;               // MFMA units (ky, seg)
  static constexpr int NWV = NT / 64;
  static constexpr int UPW = (NU + NWV - 1) / NWV;  // units per wave
  static constexpr int kRedB = NU * 16 * 64 * 4;
  static constexpr int kBiasB = NT * 4;
  static constexpr int kSmemB = (kXB + kHaloB > kRedB ? kXB + kHaloB : kRedB) + kBiasB;
  static constexpr int NH = (HR * HW + NT - 1) / NT;   // halo pixels per thread
  static_assert(kSmemB <= 160 * 1024, "fused conv1 weight gradient: LDS");
  static_assert(UPW <= 4, "fused conv1 weight gradient: accumulators");
};

// The frames' halo of the tile, loaded to registers before the data
// gradient's k-group sums (its latency hides under them): pixel (hy, hx) of
// the halo is frame pixel (2 y0 - 3 + hy, 2 x0 - 3 + hx), zero outside.
template <class F>
__device__ __forceinline__ void w1_halo_load(const SplitArgs& a, int b, int y0, int x0, int tid,
                                             float4 (&hv)[F::NH]) {
  const int H1 = 2 * a.H, W1 = 2 * a.W;
#pragma unroll
  for (int k = 0; k < F::NH; ++k) {
    const int f = tid + k * (F::NWV * 64);
    const int hy = f / F::HW, hx = f - hy * F::HW;
    const int gy = 2 * y0 - 3 + hy, gx = 2 * x0 - 3 + hx;
    hv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (f < F::HR * F::HW && (unsigned)gy < (unsigned)H1 && (unsigned)gx < (unsigned)W1)
      hv[k] = *reinterpret_cast<const float4*>(a.w1_in + (((size_t)b * H1 + gy) * W1 + gx) * 4);
  }
}

// The routing bytes of the lane's epilogue elements (split_epilogue's DGRAD
// enumeration; 4 = nothing routed, also outside the image / tile).
// Bounds-checked byte buffer loads, all issued before the first use: an
// element outside the tile / image gets an out-of-range offset (reads 0) and
// its byte is replaced by 4 after the load -- no branch per element.
template <int TM, int TN, int TX, int WK, int NWIN>
__device__ __forceinline__ void w1_route_load(const SplitArgs& a, int b, int y0, int x0, int wmi,
                                              int l31, int h, int wkg, uint8_t (&rt)[TM][16]) {
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.w1_route, (short)0, (int)(a.B * a.H * a.W * 32), 0x00020000);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      rt[i][r] = 4;
      if ((r >> 2) % WK != wkg) continue;           // (wave-uniform)
      const int m = mb + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int win = m >> 2;
      const int y = y0 + 2 * (win / (TX / 2)) + ((m >> 1) & 1);
      const int x = x0 + 2 * (win % (TX / 2)) + (m & 1);
      const bool ok = win < NWIN && y < a.H && x < a.W;
      const uint32_t off = ok ? (uint32_t)(((b * a.H + y) * a.W + x) * 32 + l31) : 0x80000000u;
      const uint8_t v = __builtin_amdgcn_raw_buffer_load_b8(rr, (int)off, 0, 0);
      rt[i][r] = ok ? v : (uint8_t)4;
    }
  }
}

// The fused conv1 weight gradient of one data-gradient tile (TN = 1, N = 32:
// channel l31).  acc: the lane's dpool1 values (split_epilogue's rows); every
// wave of the workgroup calls it (barriers inside).
template <int TY, int TX, int NT, int TM, int WK, int NWIN>
__device__ __forceinline__ void w1_tile_wgrad(const SplitArgs& a, char* smem,
                                              const f32x16 (&acc)[TM][1],
                                              const uint8_t (&rt)[TM][16],
                                              const float4 (&hv)[W1Fuse<TY, TX, NT>::NH], int b,
                                              int tile, int wmi, int l31, int h, int wkg,
                                              int tid) {
  using F = W1Fuse<TY, TX, NT>;
  const int lane = tid & 63, wid = tid >> 6;
  __bf16* X = reinterpret_cast<__bf16*>(smem);                       // [3][R][XW][32]
  __bf16* halo = reinterpret_cast<__bf16*>(smem + F::kXB);           // [HR][IROW]
  float* bsm = reinterpret_cast<float*>(smem + (F::kXB + F::kHaloB > F::kRedB
                                                    ? F::kXB + F::kHaloB : F::kRedB));
  __syncthreads();   // every wave's reads of the k-group sums (smem) are done
  // ---- the expanded image zeroed with 16-byte stores (row padding included),
  // then each element written to its routed quadrant only: 3 two-byte stores
  // an element instead of 12 with selects (conv2 data gradient 24.9 -> 24.4
  // us, same-box A/B) ----
  for (int f = tid; f < 3 * F::XPL / 8; f += NT) reinterpret_cast<u32x4*>(X)[f] = u32x4{0u, 0u, 0u, 0u};
  __syncthreads();
  float bsum = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if ((r >> 2) % WK != wkg) continue;
      const int m = mb + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int win = m >> 2;
      if (win >= NWIN) continue;                  // padding rows: no pixel
      const int ty = 2 * (win / (TX / 2)) + ((m >> 1) & 1);
      const int tx = 2 * (win % (TX / 2)) + (m & 1);
      const int q = rt[i][r];
      const float v = q < 4 ? acc[i][0][r] : 0.f;   // 4: ReLU'd window / outside the image
      bsum += v;
      __bf16 s0, s1, s2;
      split3(v, s0, s1, s2);
      if (q < 4) {
        const int e = ((2 * ty + (q >> 1)) * F::XW + 2 * tx + (q & 1)) * F::PSD + l31;
        X[e] = s0;
        X[F::XPL + e] = s1;
        X[2 * F::XPL + e] = s2;
      }
    }
  }
  // ---- the frames' halo: fp32 -> bf16 (exact), pixel stride 4 ----
#pragma unroll
  for (int k = 0; k < F::NH; ++k) {
    const int f = tid + k * NT;
    if (f < F::HR * F::HW) {
      const int hy = f / F::HW, hx = f - hy * F::HW;
      __bf16 q4[4] = {(__bf16)hv[k].x, (__bf16)hv[k].y, (__bf16)hv[k].z, (__bf16)hv[k].w};
      *reinterpret_cast<uint2*>(halo + hy * F::IROW + 4 * hx) = *reinterpret_cast<uint2*>(q4);
    }
  }
  bsm[tid] = bsum;
  __syncthreads();
  // ---- MFMAs: unit u = (ky, seg) of wave u % NWV ----
  const int gq = lane >> 4, iq = (lane & 15) >> 2, ip = lane & 3;
  const int pix0 = 8 * (gq >> 1) + iq;
  const int chn = 16 * (gq & 1) + 4 * ip;
  f32x16 wacc[F::UPW];
#pragma unroll
  for (int k = 0; k < F::UPW; ++k)
#pragma unroll
    for (int e = 0; e < 16; ++e) wacc[k][e] = 0.f;
#pragma unroll
  for (int k = 0; k < F::UPW; ++k) {
    const int u = wid + F::NWV * k;
    if (u >= F::NU) break;                        // wave-uniform
    const int ky = u / F::NSEG, seg = u - ky * F::NSEG;
    const __bf16* pa0 = X + (16 * seg + pix0) * F::PSD + chn;
    const __bf16* pb0 = halo + ky * F::IROW + 4 * (16 * seg + pix0) + chn;
#pragma unroll 4
    for (int row = 0; row < F::R; ++row) {
      bf16x8 av[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const __bf16* pa = pa0 + p * F::XPL + row * F::XW * F::PSD;
        av[p] = tr_pair(pa, pa + 4 * F::PSD);
      }
      const __bf16* pb = pb0 + row * F::IROW;
      const bf16x8 bv = tr_pair(pb, pb + 16);
      wacc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv, wacc[k], 0, 0, 0);
      wacc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv, wacc[k], 0, 0, 0);
      wacc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv, wacc[k], 0, 0, 0);
    }
  }
  __syncthreads();   // X / halo reads done: the units' tiles go where X was
  float* red = reinterpret_cast<float*>(smem);    // [NU][16][64]
#pragma unroll
  for (int k = 0; k < F::UPW; ++k) {
    const int u = wid + F::NWV * k;
    if (u >= F::NU) break;
#pragma unroll
    for (int e = 0; e < 16; ++e) red[(u * 16 + e) * 64 + lane] = wacc[k][e];
  }
  __syncthreads();
  // ---- the tile's slab: sums over the segments in order, write-through ----
  const uint32_t slab = (uint32_t)tile * 32u * (uint32_t)a.w1_np;
  const __amdgpu_buffer_rsrc_t rs =
      wt_rsrc(a.w1_part, (uint32_t)((size_t)(slab + 32u * (uint32_t)a.w1_np) * 4));
  // 16-byte stores of 4 consecutive columns (4-byte write-through stores
  // cost ~6x the time per byte, MI355X_MICROARCH.md): item = (ky, row r,
  // half h, columns 4q..4q+3 < 28)
  for (int f = tid; f < 7 * 16 * 14; f += NT) {
    const int ky = f / 224, rem = f - ky * 224;
    const int r = rem / 14, g = rem - r * 14, h2 = g / 7, q = g - h2 * 7;
    const int e = r * 64 + 32 * h2 + 4 * q;
    float4 v = *reinterpret_cast<const float4*>(red + ((ky * F::NSEG) * 16) * 64 + e);
#pragma unroll
    for (int sg = 1; sg < F::NSEG; ++sg) {
      const float4 w = *reinterpret_cast<const float4*>(red + ((ky * F::NSEG + sg) * 16) * 64 + e);
      v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
    }
    const int co = (r & 3) + 8 * (r >> 2) + 4 * h2;
    wt_store4(rs, (slab + (uint32_t)(co * a.w1_np + ky * 28 + 4 * q)) * 4, v);
  }
  if (tid < 32) {   // bias: the lanes of channel tid, waves in order
    float v = 0.f;
    for (int w = 0; w < F::NWV; ++w) v += bsm[w * 64 + tid] + bsm[w * 64 + 32 + tid];
    wt_store(rs, (slab + (uint32_t)(tid * a.w1_np + 196)) * 4, v);
  }
}

// Data-gradient epilogue through LDS: the tile's split output (the previous
// pool output's gradient, NHWC) gathered in LDS in the output's order, then
// copied out as 16-byte vectors (the accumulator layout gives 2-byte stores,
// 3 per element, scattered over the planes).  Every wave must have finished
// reading the patch / ring (the barrier at the top).  LDS: 6 TY TX N bytes.
template <int TM, int TN, int TX, int TY, int N, int WK, int NWIN, int NT>
__device__ __forceinline__ void split_epilogue_dgrad_lds(const SplitArgs& a,
                                                         const f32x16 (&acc)[TM][TN], char* smem,
                                                         int b, int y0, int x0, int wmi, int wni,
                                                         int l31, int h, int wkg, int tid) {
  constexpr int NPX = TY * TX;
  __bf16* sv = reinterpret_cast<__bf16*>(smem);   // [3][NPX][N]
  __syncthreads();
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wni * TN * 32 + 32 * j + l31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if ((r >> 2) % WK != wkg) continue;
        const int m = mb + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int win = m >> 2;
        if (win >= NWIN) continue;                // padding rows
        const int ty = 2 * (win / (TX / 2)) + ((m >> 1) & 1);
        const int tx = 2 * (win % (TX / 2)) + (m & 1);
        __bf16 hh, mm, ll;
        split3(acc[i][j][r], hh, mm, ll);
        const int e = (ty * TX + tx) * N + n;
        sv[e] = hh;
        sv[NPX * N + e] = mm;
        sv[2 * NPX * N + e] = ll;
      }
    }
  }
  __syncthreads();
  constexpr int VPP = N / 8;                      // 16-byte vectors per pixel and plane
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    __bf16* dst = a.pd_split + p * a.pd_elems;
    for (int f = tid; f < NPX * VPP; f += NT) {
      const int px = f / VPP, c = f - px * VPP;
      const int ty = px / TX, tx = px - ty * TX;
      const int y = y0 + ty, x = x0 + tx;
      if (y >= a.H || x >= a.W) continue;
      *reinterpret_cast<u32x4*>(dst + (((size_t)b * a.H + y) * a.W + x) * N + 8 * c) =
          *reinterpret_cast<const u32x4*>(sv + (p * NPX + px) * N + 8 * c);
    }
  }
}

template <int CPT, int CP, int N, int KS, int TY, int TX, int WM, int WN, int WK, bool DGRAD,
          int MF = 0>
__device__ __forceinline__ void split_conv_body(const SplitArgs& a, char* smem, int bx, int by,
                                                int bz) {
  using C = SplitCfg<CPT, CP, N, KS, TY, TX, WM, WN, WK, MF>;
  static_assert(MF == 0 || !DGRAD, "16x16x32: forward convolutions only");
  constexpr int TM = C::TM, TN = C::TN, T = C::T, NCH = C::NCH;
  __bf16* patch = reinterpret_cast<__bf16*>(smem);
  __bf16* wbuf = reinterpret_cast<__bf16*>(smem + C::kPatchB);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int z = bz, b = by;
  const int ty = bx / a.tiles_x, tx = bx % a.tiles_x;
  const int y0 = ty * TY, x0 = tx * TX;
  const __bf16* __restrict__ in = z ? a.in[1] : a.in[0];
  const __bf16* __restrict__ wk = z ? a.wk[1] : a.wk[0];
  // the bias of the lane's output channels (fwd), loaded now: at the epilogue
  // its latency was exposed once per workgroup after the last MFMA
  float bpre[C::TN * (MF ? 2 : 1)];
#pragma unroll
  for (int j = 0; j < C::TN * (MF ? 2 : 1); ++j)
    bpre[j] = DGRAD ? 0.f
                    : (z ? a.bias[1] : a.bias[0])[((wid % (WM * WN)) % WN) * C::TN * 32 +
                                                  (MF ? 16 * j + (lane & 15) : 32 * j + (lane & 31))];

  // ---- stage the halo patch of channel chunk ch (3 planes, zero outside) ----
  // Batches of 8 vectors per thread: every load of a batch is issued before
  // its LDS stores (a load -> store loop pays one memory latency per vector).
  constexpr uint32_t kOOB = 0x80000000u;
  // plane extent of the split source: (B, H, W, CPT), pooled (B, H/2, W/2, CPT) for DGRAD
  const uint32_t src_elems = DGRAD ? (uint32_t)(a.B * (a.H >> 1) * (a.W >> 1) * CPT)
                                   : (uint32_t)(a.B * a.H * a.W * CPT);
  // one descriptor over the three planes (plane p at p * in_elems), the plane
  // in the offset: a descriptor chosen per lane compiles to a waterfall loop
  // (one serialised load per distinct descriptor).  An out-of-image vector's
  // offset is kOOB (past every plane); an in-image offset never leaves its
  // own plane's src_elems.
  const __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc(
      (void*)in, (short)0, (int)((2 * (uint32_t)a.in_elems + src_elems) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rroute =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in_route, (short)0, (int)src_elems, 0x00020000);
  constexpr int NV = C::PH * C::PW * (CP / 8);             // 16-byte vectors per plane
  constexpr int NIT = (3 * NV + C::kThreads - 1) / C::kThreads;
  constexpr int BAT = NIT < 8 ? NIT : 8;
  constexpr int NIT1 = (NV + C::kThreads - 1) / C::kThreads;   // fp32 items (one per vector)
  constexpr int BAT1 = NIT1 < 4 ? NIT1 : 4;
  auto patch_load = [&](int ch, int i0, u32x4 (&v)[BAT], int (&dst)[BAT]) {
#pragma unroll
    for (int u = 0; u < BAT; ++u) {
      const int f0 = tid + (i0 + u) * C::kThreads;
      const bool live = i0 + u < NIT && f0 < 3 * NV;
      const int f = live ? f0 : 0;
      const int p = f / NV, r = f - p * NV;
      const int pix0 = r / (CP / 8), c8 = r % (CP / 8);
      // 32-channel pixels (20 or 24 dwords apart): pixels q and q + d share
      // an 8-lane store group instead of q and q + 1 (pair_rows); the block
      // of 2d pixels past the last whole one stays in order
      constexpr int NPX = C::PH * C::PW;
      const int pix = pix0 < (NPX & ~7) ? pair_rows<CP, C::CS>(pix0) : pix0;
      const int py = pix / C::PW, px = pix % C::PW;
      const int gy = y0 - a.pad + py, gx = x0 - a.pad + px;
      const bool in_img = live && (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W;
      dst[u] = live ? p * C::kPlane + py * C::RS + px * C::CS + 8 * c8 : -1;
      // bounds-checked buffer loads: outside the image (or past the
      // items) the offset is out of range and the vector reads 0 -- no
      // branch, select or 64-bit address per vector
      // (the data gradient's pooled split source, expanded through the
      // routing bytes; the forward stages fp32: stage_patch_x32)
      const uint32_t o = (uint32_t)(((b * (a.H >> 1) + (gy >> 1)) * (a.W >> 1) + (gx >> 1)) * CPT +
                                    ch * CP + 8 * c8);
      const u32x4 uw = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(rin, (int)(in_img ? (p * (uint32_t)a.in_elems + o) * 2 : kOOB), 0, 0));
      const u32x2 m = __builtin_bit_cast(
          u32x2, __builtin_amdgcn_raw_buffer_load_b64(rroute, (int)(in_img ? o : kOOB), 0, 0));
      const uint32_t q4 = ((((gy & 1) << 1) | (gx & 1))) * 0x01010101u;
      uint32_t k[4];   // bf16 pair e = channels 2e, 2e+1 (zeros route nothing)
      route_keep(m[0], q4, k[0], k[1]);
      route_keep(m[1], q4, k[2], k[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[u][e] = uw[e] & k[e];
    }
  };
  auto patch_store = [&](__bf16* buf, const u32x4 (&v)[BAT], const int (&dst)[BAT]) {
#pragma unroll
    for (int u = 0; u < BAT; ++u)
      if (dst[u] >= 0) *reinterpret_cast<u32x4*>(buf + dst[u]) = v[u];
  };
  auto stage_patch_split = [&](int ch) {   // (DGRAD)
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += BAT) {
      u32x4 v[BAT];
      int dst[BAT];
      patch_load(ch, i0, v, dst);
      patch_store(patch, v, dst);
    }
  };

  // fp32 pooled source (dgrad): a (pixel, 8-channel) item loads 32 B + its 8
  // routing bytes, keeps the routed quadrant's values, splits them (split3)
  // and stores all three planes
  auto stage_patch_f32 = [&](int ch) {
    constexpr int NI = C::PH * C::PW * (CP / 8);           // items (one per 16-byte vector)
    constexpr int NIT = (NI + C::kThreads - 1) / C::kThreads;
    constexpr int BAT = 4;
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += BAT) {
      float4 f[BAT][2];
      uint2 m[BAT];
      int dst[BAT];
      uint32_t q[BAT];
#pragma unroll
      for (int u = 0; u < BAT; ++u) {
        const int f0 = tid + (i0 + u) * C::kThreads;
        const bool live = i0 + u < NIT && f0 < NI;
        const int r = live ? f0 : 0;
        const int pix = r / (CP / 8), c8 = r % (CP / 8);
        const int py = pix / C::PW, px = pix % C::PW;
        const int gy = y0 - a.pad + py, gx = x0 - a.pad + px;
        const bool in_img = live && (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W;
        dst[u] = live ? py * C::RS + px * C::CS + 8 * c8 : -1;
        q[u] = ((gy & 1) << 1) | (gx & 1);
        f[u][0] = f[u][1] = make_float4(0.f, 0.f, 0.f, 0.f);
        m[u] = make_uint2(0x04040404u, 0x04040404u);
        if (in_img) {
          const size_t o = (((size_t)b * (a.H >> 1) + (gy >> 1)) * (a.W >> 1) + (gx >> 1)) * CPT +
                           ch * CP + 8 * c8;
          f[u][0] = *reinterpret_cast<const float4*>(a.in_f32 + o);
          f[u][1] = *reinterpret_cast<const float4*>(a.in_f32 + o + 4);
          m[u] = *reinterpret_cast<const uint2*>(a.in_route + o);
        }
      }
#pragma unroll
      for (int u = 0; u < BAT; ++u) {
        if (dst[u] < 0) continue;
        u32x4 v[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) {   // bf16 pair e = channels 2e, 2e+1
          const uint32_t mw = e < 2 ? m[u].x : m[u].y;
          const uint32_t r0 = (mw >> (16 * (e & 1))) & 0xff;
          const uint32_t r1 = (mw >> (16 * (e & 1) + 8)) & 0xff;
          const float4 fv = f[u][e >> 1];
          const float x0 = r0 == q[u] ? ((e & 1) ? fv.z : fv.x) : 0.f;
          const float x1 = r1 == q[u] ? ((e & 1) ? fv.w : fv.y) : 0.f;
          __bf16 h0, m0, l0, h1, m1, l1;
          split3(x0, h0, m0, l0);
          split3(x1, h1, m1, l1);
          v[0][e] = (uint32_t)__builtin_bit_cast(uint16_t, h0) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
          v[1][e] = (uint32_t)__builtin_bit_cast(uint16_t, m0) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, m1) << 16);
          v[2][e] = (uint32_t)__builtin_bit_cast(uint16_t, l0) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4*>(patch + p * C::kPlane + dst[u]) = v[p];
      }
    }
  };
  // forward: the fp32 activations, an (pixel, 8-channel) item = two 16-byte
  // loads, split (split_pack8) and stored as three plane vectors -- 4 bytes
  // a value through HBM instead of the 6 of a split source, and the producer
  // writes 4 instead of 6 (conv1 / conv2 forward epilogues)
  const __amdgpu_buffer_rsrc_t rin32 = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(z ? a.in32[1] : a.in32[0]), (short)0, (int)(DGRAD ? 0u : src_elems * 4), 0x00020000);
  auto stage_patch_x32 = [&](int ch) {
#pragma unroll
    for (int i0 = 0; i0 < NIT1; i0 += BAT1) {
      float4 f[BAT1][2];
      int dst[BAT1];
#pragma unroll
      for (int u = 0; u < BAT1; ++u) {
        const int f0 = tid + (i0 + u) * C::kThreads;
        const bool live = i0 + u < NIT1 && f0 < NV;
        const int r = live ? f0 : 0;
        const int pix0 = r / (CP / 8), c8 = r % (CP / 8);
        constexpr int NPX = C::PH * C::PW;
        const int pix = pix0 < (NPX & ~7) ? pair_rows<CP, C::CS>(pix0) : pix0;   // (patch_load)
        const int py = pix / C::PW, px = pix % C::PW;
        const int gy = y0 - a.pad + py, gx = x0 - a.pad + px;
        const bool in_img = live && (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W;
        dst[u] = live ? py * C::RS + px * C::CS + 8 * c8 : -1;
        const uint32_t o = (uint32_t)(((b * a.H + gy) * a.W + gx) * CPT + ch * CP + 8 * c8) * 4;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          f[u][hh] = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(rin32, (int)(in_img ? o + 16 * hh : kOOB), 0, 0));
      }
#pragma unroll
      for (int u = 0; u < BAT1; ++u) {
        if (dst[u] < 0) continue;
        u32x4 v[3];
        split_pack8(f[u][0], f[u][1], v);
#pragma unroll
        for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4*>(patch + p * C::kPlane + dst[u]) = v[p];
      }
    }
  };
  auto stage_patch = [&](int ch) {
    if constexpr (!DGRAD) stage_patch_x32(ch);
    else if (a.in_f32) stage_patch_f32(ch);
    else stage_patch_split(ch);
  };

  // ---- weights: step s = (chunk s / T, tap s % T) -> ring slot s & 1 ----
  // Two register sets: the loads of step s+2 are issued at the start of step
  // s and stored at the end of step s+1 (two steps of MFMAs to land in).
  constexpr int NSTEP = NCH * T;
  SplitWStage<C, CPT, CP, N> ws0, ws1;
  auto wload = [&](SplitWStage<C, CPT, CP, N>& w, int st) {
    const int sc = st < NSTEP ? st : NSTEP - 1;
    w.load(wk, a.wk_elems, sc / T, sc % T, tid);
  };
  stage_patch(0);
  wload(ws0, 0);
  ws0.store(wbuf, tid);
  if (NSTEP > 1) wload(ws1, 1);
  __syncthreads();
  // the tile's own pixels of the staged (split) source, for the layer's weight
  // gradient: the data gradient's expanded dconv3, the forward's Q-tower input
  // (its split is made here anyway; the stores drain under the taps' MFMAs)
  if ((DGRAD || z == 0) && NCH == 1 && a.xsplit) {
    constexpr int NV = TY * TX * (CPT / 8);
    const __amdgpu_buffer_rsrc_t rx = wt_rsrc(a.xsplit, (uint32_t)(3 * a.x_elems * 2));
#pragma unroll
    for (int i = 0; i < (3 * NV + C::kThreads - 1) / C::kThreads; ++i) {
      const int f = tid + i * C::kThreads;
      if (f < 3 * NV) {
        const int p = f / NV, r = f - p * NV;
        const int pix = r / (CPT / 8), c8 = r % (CPT / 8);
        const int ty = pix / TX, tx = pix % TX;
        const int gy = y0 + ty, gx = x0 + tx;
        if (gy < a.H && gx < a.W)
          __builtin_amdgcn_raw_buffer_store_b128(
              *reinterpret_cast<const u32x4*>(patch + p * C::kPlane + (ty + a.pad) * C::RS +
                                              (tx + a.pad) * C::CS + 8 * c8),
              rx, (int)((p * (uint32_t)a.x_elems + ((b * a.H + gy) * a.W + gx) * CPT + 8 * c8) * 2),
              0, 16);
      }
    }
  }

  // ---- per-lane operand offsets (bf16 units) ----
  const int l31 = lane & 31, h = lane >> 5;
  // wave = (k group wkg, m block wmi, n block wni); k group wkg runs k-steps
  // [wkg * KSW, +KSW) of every tap: WK x the waves on the same LDS images
  const int wkg = wid / (WM * WN), wmn = wid % (WM * WN);
  const int wmi = wmn / WN, wni = wmn % WN;
  // MF 0: row l31 of 32-row block i, channels [8 h, +8) of a 16-channel k-step;
  // MF 1: row lane & 15 of 16-row block 2 i + (half), channels [8 (lane >> 4), +8)
  // of a 32-channel k-step
  constexpr int NA = MF ? 2 * TM : TM, NB = MF ? 2 * TN : TN, KW = MF ? 32 : 16;
  const int arow = MF ? (lane & 15) : l31, koff = MF ? 8 * (lane >> 4) : 8 * h;
  int abase[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = wmi * TM * 32 + (MF ? 16 : 32) * i + arow;
    const int win = (m >> 2) < C::NWIN ? m >> 2 : 0, dy = (m >> 1) & 1, dx = m & 1;
    const int wy = win / (TX / 2), wx = win % (TX / 2);
    abase[i] = (2 * wy + dy) * C::RS + (2 * wx + dx) * C::CS + koff + KW * C::KSW * wkg;
  }
  int bbase[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j)
    bbase[j] = (wni * TN * 32 + (MF ? 16 : 32) * j + arow) * C::CW + koff + KW * C::KSW * wkg;

  f32x16 acc[TM][TN], cor[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc[i][j][r] = 0.f; cor[i][j][r] = 0.f; }
  // MF 1: the four 16x16 blocks (bi, bj) of sub-tile (i, j), elements
  // 4 (2 bi + bj) + 0..3 of acc[i][j] (f32x4 views)
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  f32x4 acc4[MF ? 2 * TM : 1][MF ? 2 * TN : 1], cor4[MF ? 2 * TM : 1][MF ? 2 * TN : 1];
  if constexpr (MF) {
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
      for (int j = 0; j < 2 * TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) { acc4[i][j][r] = 0.f; cor4[i][j][r] = 0.f; }
  }

  // The A operands (patch) of a tap's first k-step do not depend on the
  // weight ring, so they are read for tap s + 1 right after tap s's MFMAs
  // issue, before the ring's barrier; after the barrier a wave reads only its
  // B operands (the first MFMA waits for one read instead of seven of twelve,
  // and the 16 waves' post-barrier LDS burst halves).  Not across a chunk
  // edge, where the patch is restaged after the barrier.  Forward kernels
  // only: conv2 forward 25.1 -> 24.5 / 24.8 -> 24.3 us in two same-box A/Bs,
  // the step unchanged (conv3's data gradient, whose ISA is identical in
  // both builds, read 0.5 us slower in-step); with it the data gradients went
  // 24.7 -> 24.4 (conv2) and 8.2 -> 9.0 us (conv3).
  constexpr bool kPre = !DGRAD;
  bf16x8 an[3][NA];
  auto aload = [&](int s) {
    const int t = s % T, ky = t / KS, kx = t % KS;
    const __bf16* pa = patch + ky * C::RS + kx * C::CS;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < NA; ++i)
        an[p][i] = *reinterpret_cast<const bf16x8*>(pa + p * C::kPlane + abase[i]);
  };
  auto prefetched = [&](int s) { return kPre && (NCH == 1 || s % T != 0); };   // (s > 0)
  // one step: the MFMAs of tap t of the resident chunk on ring slot `slot`
  auto tap_step = [&](int s, int slot) {
    const int t = s % T;
    const __bf16* wb = wbuf + slot * 3 * C::kWSlot;
    const int ky = t / KS, kx = t % KS;
    const __bf16* pa = patch + ky * C::RS + kx * C::CS;
    const bool pre = kPre && (s == 0 || prefetched(s));
#pragma unroll
    for (int g = 0; g < C::KSW; ++g) {
      bf16x8 av[3][NA], bv[3][NB];
      if constexpr (kPre) {
#pragma unroll
        for (int j = 0; j < NB; ++j)   // in the MFMAs' order of use
#pragma unroll
          for (int p = 0; p < 3; ++p)
            bv[p][j] = *reinterpret_cast<const bf16x8*>(wb + p * C::kWSlot + bbase[j] + KW * g);
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int i = 0; i < NA; ++i)
            av[p][i] = g == 0 && pre ? an[p][i]
                                     : *reinterpret_cast<const bf16x8*>(pa + p * C::kPlane + abase[i] + KW * g);
      } else {
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
          for (int i = 0; i < NA; ++i)
            av[p][i] = *reinterpret_cast<const bf16x8*>(pa + p * C::kPlane + abase[i] + KW * g);
#pragma unroll
          for (int j = 0; j < NB; ++j)
            bv[p][j] = *reinterpret_cast<const bf16x8*>(wb + p * C::kWSlot + bbase[j] + KW * g);
        }
      }
      if constexpr (MF) {
#pragma unroll
        for (int i = 0; i < NA; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            cor4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2][i], bv[0][j], cor4[i][j], 0, 0, 0);
            cor4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[1][j], cor4[i][j], 0, 0, 0);
            cor4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[2][j], cor4[i][j], 0, 0, 0);
            cor4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[0][j], cor4[i][j], 0, 0, 0);
            cor4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[1][j], cor4[i][j], 0, 0, 0);
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], acc4[i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2][i], bv[0][j], cor[i][j], 0, 0, 0);
            cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[1][j], cor[i][j], 0, 0, 0);
            cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[2][j], cor[i][j], 0, 0, 0);
            cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0][j], cor[i][j], 0, 0, 0);
            cor[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1][j], cor[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
          }
      }
    }
    // the next tap's A operands, issued behind this tap's MFMAs
    if constexpr (kPre) {
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < NSTEP && prefetched(s + 1)) aload(s + 1);
    }
  };
  // end of step s: store step s+1's weights, restage the patch at a chunk
  // boundary (the barrier before fences every wave's reads of the old chunk)
  auto step_end = [&](SplitWStage<C, CPT, CP, N>& w, int s) {
    // keep the slot store + barrier AFTER the step's MFMAs (hipcc otherwise
    // hoists them above: every wave then waited for all its LDS reads and the
    // barrier before its first MFMA of the step)
    __builtin_amdgcn_sched_barrier(0);
    const bool chunk_edge = NCH > 1 && (s + 1) % T == 0;
    if (chunk_edge) {
      __syncthreads();
      stage_patch((s + 1) / T);
    }
    w.store(wbuf + ((s + 1) & 1) * 3 * C::kWSlot, tid);
    __syncthreads();
  };
  if (kPre) aload(0);
  for (int s = 0; s < NSTEP; s += 2) {
    if (s + 2 < NSTEP) {
      wload(ws0, s + 2);
      __builtin_amdgcn_sched_barrier(0);
    }
    tap_step(s, 0);
    if (s + 1 >= NSTEP) break;
    step_end(ws1, s);
    if (s + 3 < NSTEP) {
      wload(ws1, s + 3);
      __builtin_amdgcn_sched_barrier(0);
    }
    tap_step(s + 1, 1);
    if (s + 2 >= NSTEP) break;
    step_end(ws0, s + 1);
  }
  if constexpr (MF) {   // the 16x16 blocks into the f32x16 layout described above
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = acc4[2 * i + (g >> 1)][2 * j + (g & 1)] + cor4[2 * i + (g >> 1)][2 * j + (g & 1)];
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][4 * g + r] = v[r];
        }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += cor[i][j];
  }
  // conv2's data gradient with conv1's weight gradient fused: the frames'
  // halo and the routing bytes are loaded now, under the k-group sums
  constexpr bool kW1 = DGRAD && N == 32 && CPT == 64 && TN == 1;
  using F1 = W1Fuse<kW1 ? TY : 2, kW1 ? TX : 2, C::kThreads>;   // (no instantiation otherwise)
  float4 w1h[F1::NH];
  uint8_t w1r[TM][16];
  const bool w1 = kW1 && a.w1_part != nullptr;
  if constexpr (kW1) {
    if (w1) {
      w1_halo_load<F1>(a, b, y0, x0, tid, w1h);
      w1_route_load<TM, 1, TX, WK, C::NWIN>(a, b, y0, x0, wmi, l31, h, wkg, w1r);
    }
  }
  if (WK > 1) {
    // every k group parks its sums in LDS; group k then finishes the pooling
    // windows gi (4 accumulator rows each) with gi % WK == k, summing the
    // groups in fixed order 0..WK-1 (deterministic), so all waves share the
    // epilogue's stores
    float* red = reinterpret_cast<float*>(smem);   // one 32x32 tile per wave at a time
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        __syncthreads();                            // patch / previous tile reads done
#pragma unroll
        for (int r = 0; r < 16; ++r) red[((wkg * WM * WN + wmn) * 16 + r) * 64 + lane] = acc[i][j][r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if ((r >> 2) % WK != wkg) continue;      // (wave-uniform)
          float v = 0.f;
#pragma unroll
          for (int k = 0; k < WK; ++k) v += red[((k * WM * WN + wmn) * 16 + r) * 64 + lane];
          acc[i][j][r] = v;
        }
      }
  }
  static_assert(MF == 0 || C::NWIN * N * 7 <= C::kSmemB, "16x16x32: the LDS epilogue");
  if constexpr (!DGRAD && C::NWIN * N * 7 <= C::kSmemB) {
    split_epilogue_fwd_lds<TM, TN, TX, N, WK, C::NWIN, C::kThreads, MF>(
        a, acc, bpre, smem, b, z, y0, x0, wmi, wni, l31, h, wkg, tid);
    return;
  } else {
  if constexpr (kW1) {
    if (w1) {
      const f32x16(&acc1)[TM][1] = reinterpret_cast<const f32x16(&)[TM][1]>(acc);
      w1_tile_wgrad<TY, TX, C::kThreads, TM, WK, C::NWIN>(a, smem, acc1, w1r, w1h, b,
                                                          by * gridDim.x + bx, wmi, l31, h, wkg,
                                                          tid);
      return;
    }
  }
  if constexpr (DGRAD && 6 * TY * TX * N <= C::kSmemB) {
    if (a.pd_split && !a.pd) {
      split_epilogue_dgrad_lds<TM, TN, TX, TY, N, WK, C::NWIN, C::kThreads>(
          a, acc, smem, b, y0, x0, wmi, wni, l31, h, wkg, tid);
      return;
    }
  }
  split_epilogue<TM, TN, TX, N, DGRAD, WK, C::NWIN>(a, acc, bpre, b, z, y0, x0, wmi, wni, l31, h,
                                                    wkg);
  }
}

template <int CPT, int CP, int N, int KS, int TY, int TX, int WM, int WN, int WK, bool DGRAD,
          int MF>
__global__ __launch_bounds__(64 * WM * WN * WK) void split_conv_kernel(const SplitArgs a) {
  extern __shared__ __attribute__((aligned(16))) char sm_split[];
  split_conv_body<CPT, CP, N, KS, TY, TX, WM, WN, WK, DGRAD, MF>(a, sm_split, blockIdx.x,
                                                                     blockIdx.y, blockIdx.z);
}

template <int CPT, int CP, int N, int KS, int TY, int TX, int WM, int WN, int WK, bool DGRAD,
          int MF = 0>
inline hipError_t launch_split_conv(SplitArgs a, int nz, hipStream_t st) {
  using C = SplitCfg<CPT, CP, N, KS, TY, TX, WM, WN, WK, MF>;
  auto kern = split_conv_kernel<CPT, CP, N, KS, TY, TX, WM, WN, WK, DGRAD, MF>;
  // conv2's data gradient: room for the fused conv1 weight gradient too
  constexpr bool kW1 = DGRAD && N == 32 && CPT == 64 && C::TN == 1;
  constexpr int kW1B = kW1 ? W1Fuse<kW1 ? TY : 2, kW1 ? TX : 2, C::kThreads>::kSmemB : 0;
  constexpr int smem = C::kSmemB > kW1B ? C::kSmemB : kW1B;
  static std::atomic<uint64_t> attr{0};
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, smem))
    return e;
  // the forward epilogue writes one of the fp32 / split outputs (see
  // split_epilogue_fwd_lds)
  if (!DGRAD && ((a.out[0] && a.out_split[0]) || (a.out[1] && a.out_split[1])))
    return hipErrorInvalidValue;
  a.tiles_x = (a.W + TX - 1) / TX;
  const int tiles_y = (a.H + TY - 1) / TY;
  ddq_launch(kern, dim3(tiles_y * a.tiles_x, a.B, nz), dim3(C::kThreads), smem, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// conv1 (4 -> 32 channels, 7x7, pad 3) on the bf16 matrix cores.  Its input
// is the replay frames: integers 0..255, exact in bf16, so A has ONE plane
// and a product needs only three MFMAs (a.b0, a.b1, a.b2).  K of a kernel row
// ky = 7 taps x 4 channels, padded to 32 = two 32x32x16 k-steps; lane half h
// of step g covers taps kx = 4g + 2h, +1: two adjacent pixels x 4 channels,
// read as two ds_read_b64 from a bf16 NHWC patch (pixel stride 8 B, one zero
// column past the halo for the padded tap 7).  The 44.5 KB split weight image
// [plane][n][ky][kx 0..7][ci] (row stride 232 bf16: conflict-free b128 reads)
// is staged once per workgroup.
// ---------------------------------------------------------------------------
struct Conv1Args {
  int B, H, W, tiles_x;
  const float* in[2];          // fp32 NHWC (B,H,W,4) frames (exact integers)
  const __bf16* wk[2];         // split [n][7][8][4] (kx 7 zero)
  int64_t wk_elems;            // plane stride of the weight split tensor
  const float* bias[2];
  float* out[2];               // fp32 pooled NHWC (nullable)
  __bf16* out_split[2];        // split pooled NHWC (nullable)
  int64_t out_elems;
  uint8_t* mask[2];
};

constexpr int kConv1WPlane = 32 * 7 * 8 * 4;   // 7168 bf16 per weight plane

template <int TY, int TX, int WM>
struct Conv1Cfg {
  static constexpr int PH = TY + 6, PW = TX + 8;     // + zero column for tap 7 (+1 pad)
  static constexpr int RS0 = PW * 4;
  static constexpr int RS = RS0 + ((64 - (RS0 % 128)) + 128) % 128;   // == 64 (mod 128) bf16
  static constexpr int CW = 7 * 32 + 8;                               // 232 bf16 per n row
  static constexpr int kPatchB = PH * RS * 2;
  static constexpr int kWB = 3 * 32 * CW * 2;
  static constexpr int kSmemB = kPatchB + kWB;
  static constexpr int NWIN = TY * TX / 4;                             // padded as SplitCfg
  static constexpr int TM = (NWIN + 8 * WM - 1) / (8 * WM);
  static_assert(TM >= 1 && (WM * TM - 1) * 8 < NWIN && TX % 2 == 0 && TY % 2 == 0 && WM <= 16,
                "tile");
  static_assert(kSmemB <= 160 * 1024, "LDS");
};

// (A v_mfma_f32_16x16x32_bf16 form -- one k-step per tap row -- measured no
// faster here: conv1's MFMAs are 3 per tap row, not what bounds it.)
template <int TY, int TX, int WM>
__global__ __launch_bounds__(64 * WM) void split_conv1_kernel(const Conv1Args a) {
  using C = Conv1Cfg<TY, TX, WM>;
  constexpr int TM = C::TM;
  extern __shared__ __attribute__((aligned(16))) char sm_c1[];
  __bf16* patch = reinterpret_cast<__bf16*>(sm_c1);
  __bf16* wbuf = reinterpret_cast<__bf16*>(sm_c1 + C::kPatchB);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int z = blockIdx.z, b = blockIdx.y;
  const int ty = blockIdx.x / a.tiles_x, tx = blockIdx.x % a.tiles_x;
  const int y0 = ty * TY, x0 = tx * TX;
  const float* __restrict__ in = z ? a.in[1] : a.in[0];
  const __bf16* __restrict__ wk = z ? a.wk[1] : a.wk[0];
  constexpr int kThreads = 64 * WM;
  const float* bz_ = z ? a.bias[1] : a.bias[0];   // the epilogue's biases, early
  const float bias_pre = bz_[lane & 31];
  // patch: one pixel (4 channels) per item, fp32 -> bf16 (exact), loads first
  {
    constexpr int NP = C::PH * C::PW;
    constexpr int NIT = (NP + kThreads - 1) / kThreads;
    float4 v[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int f = tid + it * kThreads;
      const int py = f / C::PW, px = f % C::PW;
      const int gy = y0 - 3 + py, gx = x0 - 3 + px;
      v[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < NP && px < TX + 6 && (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W)
        v[it] = *reinterpret_cast<const float4*>(in + (((size_t)b * a.H + gy) * a.W + gx) * 4);
    }
    // all 3 x 7168 weight bf16 (16-byte vectors), then the stores
    constexpr int NW = 3 * kConv1WPlane / 8;
    constexpr int WIT = (NW + kThreads - 1) / kThreads;
    u32x4 w[WIT];
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int f0 = tid + it * kThreads;
      const int f = f0 < NW ? f0 : NW - 1;
      const int p = f / (kConv1WPlane / 8), r = f % (kConv1WPlane / 8);
      w[it] = *reinterpret_cast<const u32x4*>(wk + p * a.wk_elems + 8 * (size_t)r);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int f = tid + it * kThreads;
      if (f < NP) {
        const int py = f / C::PW, px = f % C::PW;
        __bf16 q[4] = {(__bf16)v[it].x, (__bf16)v[it].y, (__bf16)v[it].z, (__bf16)v[it].w};
        *reinterpret_cast<uint2*>(patch + py * C::RS + px * 4) = *reinterpret_cast<uint2*>(q);
      }
    }
#pragma unroll
    for (int it = 0; it < WIT; ++it) {
      const int f0 = tid + it * kThreads;
      const int f = f0 < NW ? f0 : NW - 1;
      const int p = f / (kConv1WPlane / 8), r = f % (kConv1WPlane / 8);
      const int n = r / 28, q8 = r % 28;        // 28 vectors of 8 per n row (7 x 8 x 4 / 8)
      *reinterpret_cast<u32x4*>(wbuf + (p * 32 + n) * C::CW + 8 * q8) = w[it];
    }
  }
  __syncthreads();
  const int l31 = lane & 31, h = lane >> 5;
  f32x16 acc[TM][1];
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wid * TM * 32 + 32 * i + l31;
    const int win = (m >> 2) < C::NWIN ? m >> 2 : 0, dy = (m >> 1) & 1, dx = m & 1;
    const int wy = win / (TX / 2), wx = win % (TX / 2);
    abase[i] = (2 * wy + dy) * C::RS + (2 * wx + dx + 2 * h) * 4;
  }
  const int bbase = l31 * C::CW + h * 8;
  f32x16 cor[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[i][0][r] = 0.f; cor[i][r] = 0.f; }
#pragma unroll
  for (int ky = 0; ky < 7; ++ky) {
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      bf16x8 bv[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bv[p] = *reinterpret_cast<const bf16x8*>(wbuf + p * 32 * C::CW + bbase + ky * 32 + 16 * g);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const __bf16* pa = patch + abase[i] + ky * C::RS + 16 * g;
        // two ds_read_b64 (2 LDS cycles each, conflict-free at RS == 64 mod
        // 128): left adjacent, hipcc merges them into one ds_read2_b64 (4 x
        // 16-lane groups on 32 banks: rows y and y+1 of a window collide,
        // 16 cycles -- 35 % of conv1's LDS cycles were conflicts)
        typedef __attribute__((address_space(3))) const u32x2 lds_u2;
        typedef __attribute__((address_space(3))) const char lds_c;
        lds_u2* la = (lds_u2*)pa;
        uint32_t hi_off = 8;                       // bytes; opaque: no merge
        asm volatile("" : "+v"(hi_off));
        const u32x2 lo = *la;
        const u32x2 hi = *(lds_u2*)((lds_c*)la + hi_off);
        u32x4 av4 = {lo[0], lo[1], hi[0], hi[1]};
        const bf16x8 av = *reinterpret_cast<bf16x8*>(&av4);
        cor[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[2], cor[i], 0, 0, 0);
        cor[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[1], cor[i], 0, 0, 0);
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[0], acc[i][0], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) acc[i][0] += cor[i];
  const float bpre[1] = {bias_pre};
  SplitArgs e{};
  e.B = a.B; e.H = a.H; e.W = a.W;
  e.out[0] = a.out[0]; e.out[1] = a.out[1];
  e.out_split[0] = a.out_split[0]; e.out_split[1] = a.out_split[1];
  e.out_elems = a.out_elems;
  e.mask[0] = a.mask[0]; e.mask[1] = a.mask[1];
  if constexpr (C::NWIN * 32 * 7 <= C::kSmemB)
    split_epilogue_fwd_lds<TM, 1, TX, 32, 1, C::NWIN, 64 * WM>(e, acc, bpre, sm_c1, b, z, y0, x0,
                                                               wid, 0, l31, h, 0, tid);
  else
    split_epilogue<TM, 1, TX, 32, false, 1, C::NWIN>(e, acc, bpre, b, z, y0, x0, wid, 0, l31, h);
}

template <int TY, int TX, int WM>
inline hipError_t launch_split_conv1(Conv1Args a, int nz, hipStream_t st, int64_t wk_elems) {
  a.wk_elems = wk_elems;
  if ((a.out[0] && a.out_split[0]) || (a.out[1] && a.out_split[1])) return hipErrorInvalidValue;
  using C = Conv1Cfg<TY, TX, WM>;
  auto kern = split_conv1_kernel<TY, TX, WM>;
  static std::atomic<uint64_t> attr{0};
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, (int)(C::kSmemB)))
    return e;
  a.tiles_x = (a.W + TX - 1) / TX;
  const int tiles_y = (a.H + TY - 1) / TY;
  ddq_launch(kern, dim3(tiles_y * a.tiles_x, a.B, nz), dim3(64 * WM), C::kSmemB, st, a);
  return hipGetLastError();
}

}  // namespace ddq
