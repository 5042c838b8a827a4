// conv2 / conv3 weight gradient on the bf16 matrix cores, fp32-exact split
// operands (split.h), in the row-streaming form of wgradd.h.
//
// dW[co][ky][kx][ci] = sum_{b,y,x} dconv[b][y][x][co] * in[b][y+ky-P][x+kx-P][ci]
// db[co]             = sum_{b,y,x} dconv[b][y][x][co]
//
// A workgroup owns one (co block cb, tap row ky) pair -- KS x CIN/32 output
// tiles of 32 x 32 -- over a group of image rows; each of its 4 waves streams
// its own rows through a private LDS region: the input row y+ky-P (3 bf16
// planes, zero halo) and the cb block of the dconv row (3 planes, expanded
// from the pooled split gradient through the pool's routing bytes).  One
// 32x32x16 k-step = 16 pixels of the row; both operands are read pixel-major
// out of their NHWC rows with ds_read_b64_tr_b16 (a 16-lane group reads 4
// pixels x 16 channels and each lane receives its channel's 4 pixels), so the
// kx shift of the input operand is just another row address: no im2col, no
// shifted copies.  6 MFMAs per (tile, k-step), small products first, into one
// fp32 accumulator.  The waves' tiles are summed in LDS
// in fixed order and stored as the group's fp32 slab in the wgrad reducer's
// layout ([group][co][NP], bias at n = KC; deterministic, no atomics).  The
// bias column is summed on the VALU (fp32, from the staged split values) by
// the ky == 0 workgroups.
#pragma once
#include "split.h"

namespace ddq {

// Row groups (= slabs) of a weight gradient over `rows` image rows: about
// `target` workgroups over the nts (co block, tap row) pairs, whole XCD
// rounds (the kernels' decode deals a group's workgroups to one XCD).
inline void wgrads_groups(int rows, int nts, int* G, int* RPG, int target = 512) {
  int g = target / nts;
  if (g >= 16) g &= ~7;
  if (g < 1) g = 1;
  if (g > rows) g = rows;
  const int rpg = (rows + g - 1) / g;
  *RPG = rpg;
  *G = (rows + rpg - 1) / rpg;
}


struct WgradSArgs {
  int B, H, W;              // layer grid (input and dconv share H x W)
  int G, RPG;               // row groups (= slabs) and rows per group
  int NP;                   // slab pitch
  const __bf16* in;         // split NHWC (B,H,W,CIN), plane stride in_elems
  int64_t in_elems;
  const __bf16* dpool;      // split pooled gradient (B,H/2,W/2,COUT), plane stride d_elems
  int64_t d_elems;
  const uint8_t* droute;    // its NHWC routing bytes
  float* part;              // [G][COUT][NP]
  const float* dpool_f32;   // DSRC 1: the pooled gradient in fp32 instead
                            // (split while staged)
  const __bf16* dfull;      // DSRC 2: the gradient already expanded and split,
                            // NHWC (B,H,W,COUT), plane stride d_elems (conv3's:
                            // a side output of its data gradient's staging)
};

// LDS geometry of one wave's region (bf16 units).  Pixel strides keep the
// transposed reads conflict-free: a 32-lane half reads 4 pixels x 32 channels
// = 4 x 64 B; pixel stride == 16 banks (mod 64) puts them on 64 distinct banks.
template <int CIN, int PAD>
struct WgradSGeom {
  static constexpr int PSI = CIN == 32 ? 32 : 96;   // input pixel stride (64 B / 192 B)
  static constexpr int PSD = 32;                    // dconv pixel stride (64 B)
  // k-steps cover 16 pixels: rows are sized to W rounded up to 16, the dconv
  // tail pixels stay zero (never written), the input halo / tail likewise
  static __host__ __device__ int w16(int W) { return (W + 15) & ~15; }
  static __host__ __device__ int in_plane(int W) { return (w16(W) + 2 * PAD + 8) * PSI; }
  static __host__ __device__ int d_plane(int W) { return w16(W) * PSD; }
  static __host__ __device__ int region(int W) { return 3 * (in_plane(W) + d_plane(W)); }
};



// DSRC: the dconv rows' source -- 0: pooled split + routing bytes (conv2's),
// 1: pooled fp32 + routing bytes, split while staged, 2: expanded split
// (dfull: pure 16-byte copies, no VALU per element)
template <int CIN, int COUT, int KS, int PAD, int WMAX, int DSRC>
__device__ __forceinline__ void wgrads_body(const WgradSArgs& a, char* smem, int L) {
  constexpr bool DF32 = DSRC == 1;
  constexpr int NCB = CIN / 32;
  constexpr int T = KS * NCB;
  constexpr int KC = KS * KS * CIN;
  using Geo = WgradSGeom<CIN, PAD>;
  const int W = a.W, H = a.H;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ipl = Geo::in_plane(W), dpl = Geo::d_plane(W);
  __bf16* rin = reinterpret_cast<__bf16*>(smem) + w * Geo::region(W);   // [3][W+2P+8][PSI]
  __bf16* rd = rin + 3 * ipl;                                            // [3][W][PSD]
  // XCD-aware decode (as wgradd): every (cb, ky) workgroup of row group g
  // gets the same L % 8, so the group's rows stay in one XCD's L2
  constexpr int NTS = (COUT / 32) * KS;
  const int xcd = L & 7, q = L >> 3;
  const int ts = q % NTS, g = xcd + 8 * (q / NTS);
  if (g >= a.G) return;
  const int cb = ts / KS, ky = ts % KS;
  const int r0 = g * a.RPG;
  const int r1 = min(a.B * H, r0 + a.RPG);

  // zero the pixels rows never write: the input halo / tail, the dconv tail
  {
    // only the halo / tail pixels (x < PAD, x >= W + PAD), compile-time
    // divisors: walking every pixel with runtime divisions cost ~1500 VALU a
    // wave, more than conv3's MFMAs of a wave's rows
    constexpr int CPV = Geo::PSI / 8;
    const int nh = Geo::w16(W) + 2 * PAD + 8 - W;   // halo + tail pixels of a row
#pragma unroll
    for (int p = 0; p < 3; ++p)
      for (int i = lane; i < nh * CPV; i += 64) {
        const int hx = i / CPV, c = i % CPV;
        const int x = hx < PAD ? hx : hx + W;
        reinterpret_cast<u32x4*>(rin + p * ipl + x * Geo::PSI)[c] = u32x4{0u, 0u, 0u, 0u};
      }
    for (int i = lane; i < 3 * (Geo::w16(W) - W) * (Geo::PSD / 8); i += 64) {
      const int per = (Geo::w16(W) - W) * (Geo::PSD / 8);
      const int p = i / per, r = i - p * per;
      reinterpret_cast<u32x4*>(rd + p * dpl + W * Geo::PSD)[r] = u32x4{0u, 0u, 0u, 0u};
    }
  }

  // one fp32 accumulator per tile for all six products (2 waves per SIMD
  // need <= 256 registers; a separate correction accumulator took 80-96 more).
  // Six MFMA roundings per 16 K, against sixteen (one per product) on the
  // f32-input MFMA path this replaces.
  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // channels 8*(lane&3) + j of cb

  // ---- row staging: global -> registers (issued ahead), registers -> LDS ----
  // Every lane keeps one 8-channel chunk and walks the pixels (no division
  // in the loops: a runtime-divisor mapping of the vectors cost ~600 VALU per
  // row, 10x the MFMAs).  Input: CC chunks per pixel, 64 / CC pixels a pass;
  // pooled dconv: 4 chunks of the 32-channel block, 16 pooled pixels a pass,
  // one routing load per pixel chunk for the three planes.
  constexpr int CC = CIN / 8, PPP = 64 / CC;
  constexpr int NPI = (WMAX + PPP - 1) / PPP;
  // dconv chunks per lane: pooled pixels (16 a pass), or DSRC 2 full-width pixels
  constexpr int NPD = DSRC == 2 ? (WMAX + 15) / 16 : (WMAX / 2 + 15) / 16;
  const int ic8 = lane % CC, ipx = lane / CC;
  const int dc8 = lane & 3, dpx = lane >> 2;
  struct Regs {
    u32x4 i[3][NPI];
    u32x4 d[3][NPD];
    float4 f[2][NPD];    // DF32: the 8 fp32 values of the chunk
    u32x2 m[NPD];
  };
  // Every load is issued unconditionally as a bounds-checked buffer load: an
  // out-of-range vector gets the offset kOOB and reads 0, so there is no
  // select after the load and no 64-bit address math (the loads used to be
  // clamped to element 0 and zeroed with v_cndmask).  With no branches
  // around them the compiler counts a row set's loads exactly and waits for
  // that set only.  The row's (image, y) advance by the wave stride without
  // a runtime division (H >= 8 > 4).
  constexpr uint32_t kOOB = 0x80000000u;
  const uint32_t ib = (uint32_t)(a.in_elems * 2);
  const __amdgpu_buffer_rsrc_t rin_g[3] = {
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in, (short)0, (int)ib, 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.in + a.in_elems), (short)0, (int)ib, 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.in + 2 * a.in_elems), (short)0, (int)ib,
                                        0x00020000)};
  // elements of a plane of the dconv source
  const uint32_t db = DSRC == 2 ? (uint32_t)(a.B * H * W * COUT)
                                : (uint32_t)(a.B * (H >> 1) * (W >> 1) * COUT);
  const __bf16* dsp = DSRC == 2 ? a.dfull : a.dpool;
  const __amdgpu_buffer_rsrc_t rd_g[3] = {
      __builtin_amdgcn_make_buffer_rsrc((void*)(DF32 ? (const void*)a.dpool_f32 : (const void*)dsp),
                                        (short)0, (int)(DF32 ? db * 4 : db * 2), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)(DF32 ? nullptr : dsp + a.d_elems), (short)0,
                                        (int)(db * 2), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc((void*)(DF32 ? nullptr : dsp + 2 * a.d_elems), (short)0,
                                        (int)(db * 2), 0x00020000)};
  const __amdgpu_buffer_rsrc_t rm_g =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.droute, (short)0, (int)db, 0x00020000);
  int lb = (r0 + w) / H, ly = (r0 + w) - lb * H;   // (image, y) of the next row to load
  auto load = [&](Regs& R, int row) {
    const bool live = row < r1;
    const int yi = ly + ky - PAD;
    const bool vin = live && (unsigned)yi < (unsigned)H;
    const uint32_t i0 = (uint32_t)(((lb * H + yi) * W + ipx) * CIN + 8 * ic8);
#pragma unroll
    for (int u = 0; u < NPI; ++u) {
      const bool ok = vin && ipx + u * PPP < W;
      const uint32_t o = ok ? (i0 + (uint32_t)(u * PPP * CIN)) * 2 : kOOB;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        R.i[p][u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rin_g[p], (int)o, 0, 0));
    }
    if (DSRC == 2) {   // expanded split rows: 16-byte copies
      const uint32_t o0 = (uint32_t)(((lb * H + ly) * W + dpx) * COUT + cb * 32 + 8 * dc8);
#pragma unroll
      for (int u = 0; u < NPD; ++u) {
        const bool ok = live && dpx + 16 * u < W;
        const uint32_t o = o0 + (uint32_t)(u * 16 * COUT);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          R.d[p][u] = __builtin_bit_cast(
              u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd_g[p], (int)(ok ? o * 2 : kOOB), 0, 0));
      }
      ly += 4;
      if (ly >= H) { ly -= H; ++lb; }
      return;
    }
    const uint32_t o0 =
        (uint32_t)(((lb * (H >> 1) + (ly >> 1)) * (W >> 1) + dpx) * COUT + cb * 32 + 8 * dc8);
#pragma unroll
    for (int u = 0; u < NPD; ++u) {
      const bool ok = live && dpx + 16 * u < (W >> 1);
      const uint32_t o = ok ? o0 + (uint32_t)(u * 16 * COUT) : 0u;
      // routing bytes past the range read 0: the values there read 0 as well
      R.m[u] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rm_g, (int)(ok ? o : kOOB), 0, 0));
      if (DF32) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          R.f[hh][u] = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(rd_g[0], (int)(ok ? (o + 4 * hh) * 4 : kOOB), 0, 0));
      } else {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          R.d[p][u] = __builtin_bit_cast(
              u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd_g[p], (int)(ok ? o * 2 : kOOB), 0, 0));
      }
    }
    ly += 4;
    if (ly >= H) { ly -= H; ++lb; }
  };
  auto store = [&](Regs& R, int row) {
    const uint32_t qy = (row & 1) << 1;   // H is even: row and y have one parity
    if (DF32) {   // split the fp32 chunk into the three planes (split.h split3)
#pragma unroll
      for (int u = 0; u < NPD; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float x0 = e < 2 ? (e == 0 ? R.f[0][u].x : R.f[0][u].z)
                                 : (e == 2 ? R.f[1][u].x : R.f[1][u].z);
          const float x1 = e < 2 ? (e == 0 ? R.f[0][u].y : R.f[0][u].w)
                                 : (e == 2 ? R.f[1][u].y : R.f[1][u].w);
          __bf16 h0, m0, l0, h1, m1, l1;
          split3(x0, h0, m0, l0);
          split3(x1, h1, m1, l1);
          R.d[0][u][e] = (uint32_t)__builtin_bit_cast(uint16_t, h0) |
                         ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
          R.d[1][u][e] = (uint32_t)__builtin_bit_cast(uint16_t, m0) |
                         ((uint32_t)__builtin_bit_cast(uint16_t, m1) << 16);
          R.d[2][u][e] = (uint32_t)__builtin_bit_cast(uint16_t, l0) |
                         ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
        }
    }
#pragma unroll
    for (int u = 0; u < NPI; ++u)
      if (ipx + u * PPP < W)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<u32x4*>(rin + p * ipl + (ipx + u * PPP + PAD) * Geo::PSI + 8 * ic8) =
              R.i[p][u];
    if (DSRC == 2) {
#pragma unroll
      for (int u = 0; u < NPD; ++u) {
        const int px = dpx + 16 * u;
        if (px >= W) continue;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          *reinterpret_cast<u32x4*>(rd + p * dpl + px * Geo::PSD + 8 * dc8) = R.d[p][u];
          if (ky == 0) {   // bias: fp32 value = sum of the three planes
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bsum[2 * e] += __builtin_bit_cast(float, R.d[p][u][e] << 16);
              bsum[2 * e + 1] += __builtin_bit_cast(float, R.d[p][u][e] & 0xffff0000u);
            }
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < (DSRC == 2 ? 0 : NPD); ++u) {
      const int px = dpx + 16 * u;
      if (px >= (W >> 1)) continue;
#pragma unroll
      for (int d2 = 0; d2 < 2; ++d2) {
        // odd pooled pixels write their two expanded pixels in the other order:
        // an 8-lane ds_write_b128 group (pooled pixels p, p + 1) then writes
        // pixels 16 / 48 dwords apart, not 32 (banks (a/4) mod 32: conflict-free)
        const int dx = d2 ^ (dpx & 1);
        const uint32_t qd = qy | dx;
        // per bf16 pair e (channels 2e, 2e+1): keep-masks from the routing bytes
        uint32_t keep[4];
        route_keep(R.m[u][0], qd * 0x01010101u, keep[0], keep[1]);
        route_keep(R.m[u][1], qd * 0x01010101u, keep[2], keep[3]);
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = R.d[p][u][e] & keep[e];
          *reinterpret_cast<u32x4*>(rd + p * dpl + (2 * px + dx) * Geo::PSD + 8 * dc8) = o;
          if (ky == 0) {   // bias: fp32 value = sum of the three planes
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              bsum[2 * e] += __builtin_bit_cast(float, o[e] << 16);
              bsum[2 * e + 1] += __builtin_bit_cast(float, o[e] & 0xffff0000u);
            }
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // per-lane transposed-read offsets: group gq = lane >> 4 reads pixel rows
  // 8*(gq>>1) + {0..3} / {4..7}, channels 16*(gq&1) + 4*(lane&3) of a 32 block
  const int gq = lane >> 4, iq = (lane & 15) >> 2, ip = lane & 3;
  const int pix0 = 8 * (gq >> 1) + iq;
  const int chn = 16 * (gq & 1) + 4 * ip;
  auto compute = [&]() {
#pragma unroll
    for (int s = 0; s < WMAX / 16; ++s) {
      if (16 * s >= W) break;
      // the A fragments, then the B fragments one kx ahead of their MFMAs
      // (all of them live at once took the registers of a second row set)
      bf16x8 av[3], bv[2][NCB][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const __bf16* pa = rd + p * dpl + (16 * s + pix0) * Geo::PSD + chn;
        av[p] = tr_pair(pa, pa + 4 * Geo::PSD);
      }
      auto bload = [&](int kx) {
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const __bf16* pb = rin + p * ipl + (16 * s + pix0 + kx) * Geo::PSI + 32 * c + chn;
            bv[kx & 1][c][p] = tr_pair(pb, pb + 4 * Geo::PSI);
          }
      };
      bload(0);
#pragma unroll
      for (int kx = 0; kx < KS; ++kx) {
        if (kx + 1 < KS) bload(kx + 1);
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          const int t = kx * NCB + c;
          const bf16x8* b = bv[kx & 1][c];
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], b[0], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], b[1], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], b[2], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], b[0], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], b[1], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], b[0], acc[t], 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  };

  {   // one register set: the next row's loads are issued right after this
      // row's LDS stores and land under its MFMAs (a second set, loading two
      // rows ahead, measured no faster: the kernel is not waiting on them)
    Regs g;
    int row = r0 + w;
    if (row < r1) load(g, row);
    for (; row < r1; row += 4) {
      store(g, row);
      load(g, row + 4);             // rows past r1 read nothing (live = false)
      __builtin_amdgcn_sched_barrier(0);
      compute();
    }
  }

  // ---- sum the four waves' tiles in fixed order, store the group slab ----
  float* red = reinterpret_cast<float*>(smem);        // [4 waves][16 r][64 lanes]
  // slab stores write-through (wt_store): the reduce reads them from memory
  // anyway, and the kernel's end then has no dirty slab lines to write back
  const __amdgpu_buffer_rsrc_t srs = wt_rsrc(a.part, (uint32_t)((size_t)a.G * COUT * a.NP * 4));
  const uint32_t sbase = (uint32_t)(((size_t)g * COUT + (size_t)cb * 32) * a.NP * 4);
#pragma unroll
  for (int t = 0; t < T; ++t) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc[t][r];
    __syncthreads();
    const int nbase = (ky * KS + t / NCB) * CIN + (t % NCB) * 32;
    {   // thread = (tile row r, lanes 4q..4q+3): 4 consecutive columns, one
        // 16-byte write-through store (4-byte ones cost ~6x per byte)
      const int tt = threadIdx.x, r = tt >> 4, l0 = 4 * (tt & 15);
      const int e = r * 64 + l0;
      const float4 a0 = *reinterpret_cast<const float4*>(red + e);
      const float4 a1 = *reinterpret_cast<const float4*>(red + 1024 + e);
      const float4 a2 = *reinterpret_cast<const float4*>(red + 2048 + e);
      const float4 a3 = *reinterpret_cast<const float4*>(red + 3072 + e);
      const float4 v = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                                   (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
      const int co = (r & 3) + 8 * (r >> 2) + 4 * (l0 >> 5);
      wt_store4(srs, sbase + (uint32_t)((co * a.NP + nbase + (l0 & 31)) * 4), v);
    }
  }
  if (ky == 0) {   // bias column n = KC: lanes with equal lane & 3 share 8 channels
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[(w * 64 + lane) * 8 + j] = bsum[j];
    __syncthreads();
    if (threadIdx.x < 32) {
      const int co = threadIdx.x, c8 = co >> 3, j = co & 7;
      float v = 0.f;
      for (int ww = 0; ww < 4; ++ww)
        for (int l = c8; l < 64; l += 4) v += red[(ww * 64 + l) * 8 + j];
      wt_store(srs, sbase + (uint32_t)((co * a.NP + KC) * 4), v);
    }
  }
}

template <int CIN, int PAD>
inline size_t wgrads_smem_bytes(int W) {
  const size_t f = (size_t)4 * WgradSGeom<CIN, PAD>::region(W) * 2;
  return f > 4 * 16 * 64 * 4 + 0 ? f : 4 * 16 * 64 * 4;   // >= the 4-wave reduction image
}

// Two weight gradients in one launch (conv2's and conv3's: both need only the
// data gradient conv3's data-gradient launch wrote): blocks [0, n0) are the
// first's, the rest the second's -- one kernel boundary fewer, and the second's
// workgroups fill the CUs the first's tail leaves idle.  n0 is a multiple of 8,
// so each keeps its XCD-aware decode.  LDS: the larger of the two.  Two waves
// per SIMD (<= 256 registers): the other wave's MFMAs cover each wave's row
// staging and LDS round trips.
template <int CIN0, int COUT0, int KS0, int PAD0, int WMAX0, int DSRC0, int CIN1, int COUT1,
          int KS1, int PAD1, int WMAX1, int DSRC1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void wgrads_pair_kernel(
    const WgradSArgs a0, const WgradSArgs a1, int n0) {
  extern __shared__ __attribute__((aligned(16))) char sm_wgp[];
  if ((int)blockIdx.x < n0)
    wgrads_body<CIN0, COUT0, KS0, PAD0, WMAX0, DSRC0>(a0, sm_wgp, blockIdx.x);
  else
    wgrads_body<CIN1, COUT1, KS1, PAD1, WMAX1, DSRC1>(a1, sm_wgp, blockIdx.x - n0);
}

template <int CIN0, int COUT0, int KS0, int PAD0, int WMAX0, int DSRC0, int CIN1, int COUT1,
          int KS1, int PAD1, int WMAX1, int DSRC1>
inline hipError_t launch_wgrads_pair_w(const WgradSArgs& a0, const WgradSArgs& a1, hipStream_t st) {
  const size_t s0 = wgrads_smem_bytes<CIN0, PAD0>(a0.W), s1 = wgrads_smem_bytes<CIN1, PAD1>(a1.W);
  const size_t shm = s0 > s1 ? s0 : s1;
  if (shm > 160 * 1024) return hipErrorInvalidValue;
  auto kern = wgrads_pair_kernel<CIN0, COUT0, KS0, PAD0, WMAX0, DSRC0, CIN1, COUT1, KS1, PAD1,
                                 WMAX1, DSRC1>;
  static std::atomic<uint64_t> attr{0};
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, (int)(160 * 1024)))
    return e;
  const int n0 = (a0.G + 7) / 8 * 8 * (COUT0 / 32) * KS0;
  const int n1 = (a1.G + 7) / 8 * 8 * (COUT1 / 32) * KS1;
  ddq_launch(kern, dim3(n0 + n1), dim3(256), shm, st, a0, a1, n0);
  return hipGetLastError();
}

// conv2's (on the split pooled dpool2) + conv3's (on the expanded split
// dconv3); the staging registers are sized for the widest row of each
inline hipError_t launch_wgrads_conv23(const WgradSArgs& a2, const WgradSArgs& a3, hipStream_t st) {
  if (a2.W <= 16) return launch_wgrads_pair_w<32, 64, 5, 2, 16, 0, 64, 64, 3, 1, 16, 2>(a2, a3, st);
  if (a2.W <= 32) return launch_wgrads_pair_w<32, 64, 5, 2, 32, 0, 64, 64, 3, 1, 16, 2>(a2, a3, st);
  if (a2.W <= 64) return launch_wgrads_pair_w<32, 64, 5, 2, 64, 0, 64, 64, 3, 1, 32, 2>(a2, a3, st);
  return hipErrorInvalidValue;   // frames > 128: not supported
}

}  // namespace ddq


