// conv2 / conv3 weight gradient, direct form (gfx950).
//
// dW[co][ky][kx][ci] = sum_{b,y,x} dconv[b][y][x][co] * in[b][y+ky-P][x+kx-P][ci]
// db[co]             = sum_{b,y,x} dconv[b][y][x][co]
//
// The implicit-GEMM form re-derives (b, y, x, ky, kx, ci) for every staged
// operand (8-15 VALU per MFMA measured).  Here a workgroup owns one
// (co block cb, tap row ky) pair -- KS x CIN/32 output tiles of 32 x 32
// (tile (kx, cib) = columns n = (ky*KS + kx)*CIN + cib*32 + 0..31) -- over a
// contiguous group of image rows.  Each wave streams its own rows through a
// private LDS region: the input row y+ky-P (with a zero halo of P pixels) and
// the cb block of the dconv row.  One MFMA k-step covers the pixel pair
// (2s, 2s+1): the dconv operand is read once and feeds every tile of the
// wave (KS*CIN/32 MFMAs per ds_read of A, one ds_read of B each), so the
// inner loop is pure LDS->MFMA with no index math.  The bias column is
// summed on the VALU from the staged dconv rows by the ky == 0 workgroups.
// At the end the four waves' accumulators are summed through LDS (fixed
// order, deterministic) and stored as the group's fp32 slab in the wgrad
// reducer's layout ([group][co][n], bias at n = KC).
#pragma once
#include "common.h"

namespace ddq {

struct WgradDArgs {
  int B, H, W;              // layer grid (input and dconv share H x W)
  int G, RPG;               // row groups (= slabs) and rows per group
  int NP;                   // slab pitch
  const float* dconv;       // NHWC (B,H,W,COUT); PSRC: pooled (B,H/2,W/2,COUT)
  const float* in;          // NHWC (B,H,W,CIN)
  float* part;              // [G][COUT][NP]
  const uint8_t* droute;    // PSRC: NHWC routing bytes of the pooled gradient
};

template <int CIN, int PAD>
struct WgradDGeom {
  // floats of one wave's LDS region for width W
  static __host__ __device__ int in_floats(int W) { return (((W + 2 * PAD + 1) * CIN) + 3) & ~3; }
  static __host__ __device__ int region(int W) { return in_floats(W) + ((W + 1) >> 1) * 64; }
};

// PSRC: dconv is given pooled (the gradient of the 2x2 max-pool output plus
// its routing bytes, as fc4's data gradient leaves it) and expanded while the
// rows are staged: value at the routed quadrant, 0 at the other three.
// Body of one 4-wave workgroup L of the 1-D grid (a fused launch with wider
// workgroups ends the extra waves first; s_barrier does not wait for them).
template <int CIN, int COUT, int KS, int PAD, bool PSRC>
__device__ __forceinline__ void wgradd_body(const WgradDArgs& a, float* sm, int L) {
  constexpr int NCB = CIN / 32;
  constexpr int T = KS * NCB;
  constexpr int KC = KS * KS * CIN;
  using Geo = WgradDGeom<CIN, PAD>;
  const int W = a.W, H = a.H;
  const int W2 = (W + 1) >> 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int inf = Geo::in_floats(W);
  float* rin = sm + w * Geo::region(W);     // input row, pixel 0 <-> x = -PAD
  float* rd = rin + inf;                    // dconv row, [x][32] of block cb
  // XCD-aware decode of the 1-D grid: workgroups are dealt to the 8 XCDs
  // round-robin, so give every (cb, ky) workgroup of row group g the same
  // L % 8 and the group's rows stay in one XCD's L2.
  constexpr int NTS = (COUT / 32) * KS;
  const int xcd = L & 7, q = L >> 3;
  const int ts = q % NTS, g = xcd + 8 * (q / NTS);
  if (g >= a.G) return;
  const int cb = ts / KS, ky = ts % KS;
  const int r0 = g * a.RPG;
  const int r1 = min(a.B * H, r0 + a.RPG);

  // zero halo columns (never overwritten) and the odd-width tail pixel
  for (int i = lane; i < PAD * CIN; i += 64) rin[i] = 0.f;
  for (int i = lane; i < (PAD + 1) * CIN; i += 64) rin[(PAD + W) * CIN + i] = 0.f;
  if (W & 1)
    for (int i = lane; i < 32; i += 64) rd[W * 32 + i] = 0.f;

  f32x16 acc[T];
  float4 bsum = f4zero();                   // bias: lane sums channels 4*(lane&7).. of block cb
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // Row staging: a wave moves W*CIN/4 + W*8 float4 per row through bounds-
  // checked buffer loads (out-of-range rows / halo rows read as 0 with no
  // branch).  When both fit one 64-lane x 4 batch (S <= 64) the next row's
  // loads are issued before the current row's MFMAs from a second register
  // set (rows unrolled by two so no copies force an early vmcnt wait);
  // otherwise rows are staged synchronously in 4-deep batches.
  const int nin = W * CIN / 4, nd = W * 8;
  const int rows_total = a.B * H;
  const __amdgpu_buffer_rsrc_t rs_in =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in, (short)0, rows_total * W * CIN * 4, 0x00020000);
  const int dsz = PSRC ? (rows_total / 2) * (W / 2) * COUT : rows_total * W * COUT;
  const __amdgpu_buffer_rsrc_t rs_d =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dconv, (short)0, dsz * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_m =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.droute, (short)0, PSRC ? dsz : 0, 0x00020000);
  constexpr int kOOB = 0x7ff00000;   // beyond any tensor here: reads 0
  struct Regs { float4 i[4], d[4]; uint32_t m[4]; };
  auto load = [&](Regs& g, int row, int base) {
    const int b = row / H, yi = row - b * H + ky - PAD;
    const bool vin = (unsigned)yi < (unsigned)H && row < rows_total;
    const int ib = vin ? (b * H + yi) * W * CIN * 4 : kOOB;
    // PSRC: pooled row (b, y/2) of width W/2
    const int db = row >= rows_total ? kOOB
                   : PSRC ? ((b * (H >> 1) + ((row - b * H) >> 1)) * (W >> 1) * COUT + cb * 32) * 4
                          : (row * W * COUT + cb * 32) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + lane + 64 * j;
      const int oi = i < nin ? ib + i * 16 : kOOB;
      const int px = PSRC ? (i >> 4) : (i >> 3);
      const int od = i < nd ? db + (px * COUT + (i & 7) * 4) * 4 : kOOB;
      auto vi = __builtin_amdgcn_raw_buffer_load_b128(rs_in, oi, 0, 0);
      auto vd = __builtin_amdgcn_raw_buffer_load_b128(rs_d, od, 0, 0);
      g.i[j] = *reinterpret_cast<float4*>(&vi);
      g.d[j] = *reinterpret_cast<float4*>(&vd);
      if (PSRC) g.m[j] = __builtin_amdgcn_raw_buffer_load_b32(rs_m, od == kOOB ? kOOB : od >> 2, 0, 0);
    }
  };
  auto store = [&](const Regs& g, int base, int row) {
    float4* dst = reinterpret_cast<float4*>(rin + PAD * CIN);
    float4* dd = reinterpret_cast<float4*>(rd);
    const uint32_t qy = PSRC ? (((row - (row / H) * H) & 1) << 1) : 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = base + lane + 64 * j;
      if (i < nin) dst[i] = g.i[j];
      if (i < nd) {
        float4 d = g.d[j];
        if (PSRC) {
          const uint32_t q = qy | ((i >> 3) & 1), m = g.m[j];
          d.x = (m & 0xff) == q ? d.x : 0.f;
          d.y = ((m >> 8) & 0xff) == q ? d.y : 0.f;
          d.z = ((m >> 16) & 0xff) == q ? d.z : 0.f;
          d.w = (m >> 24) == q ? d.w : 0.f;
        }
        dd[i] = d;
        bsum.x += d.x; bsum.y += d.y; bsum.z += d.z; bsum.w += d.w;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // ---- MFMA: k-step s = pixels (2s, 2s+1); lane half h takes pixel 2s+h ----
  // The KS input pixels of step s are a window that slides by two pixels per
  // step: keep it in registers, load only the two new pixels (and the next
  // dconv value) per step, and issue those loads before this step's MFMAs
  // (pinned by a scheduling barrier) -- the plain load/wait/MFMA loop left
  // three LDS round trips exposed per step.
  auto compute = [&]() {
    const float* pa = rd + h * 32 + l31;
    const float* pb = rin + h * CIN + l31;
    float bw[KS][NCB];
    float av = pa[0];
#pragma unroll
    for (int kx = 0; kx < KS; ++kx)
#pragma unroll
      for (int c = 0; c < NCB; ++c) bw[kx][c] = pb[kx * CIN + c * 32];
    for (int s = 0; s < W2; ++s) {
      float an = 0.f, n0[NCB], n1[NCB];
      const bool more = s + 1 < W2;
      if (more) {
        an = pa[(s + 1) * 64];
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          n0[c] = pb[(2 * s + KS) * CIN + c * 32];
          n1[c] = pb[(2 * s + KS + 1) * CIN + c * 32];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kx = 0; kx < KS; ++kx)
#pragma unroll
        for (int c = 0; c < NCB; ++c)
          acc[kx * NCB + c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bw[kx][c],
                                                                  acc[kx * NCB + c], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (more) {
#pragma unroll
        for (int kx = 0; kx + 2 < KS; ++kx)
#pragma unroll
          for (int c = 0; c < NCB; ++c) bw[kx][c] = bw[kx + 2][c];
#pragma unroll
        for (int c = 0; c < NCB; ++c) {
          bw[KS - 2][c] = n0[c];
          bw[KS - 1][c] = n1[c];
        }
        av = an;
      }
    }
    __builtin_amdgcn_wave_barrier();
  };

  if (nin <= 256 && nd <= 256) {
    Regs ga, gb;
    int row = r0 + w;
    if (row < r1) load(ga, row, 0);
    for (; row < r1; row += 8) {
      store(ga, 0, row);
      load(gb, row + 4, 0);          // rows past r1 only read (bounded), never staged
      compute();
      if (row + 4 >= r1) break;
      store(gb, 0, row + 4);
      load(ga, row + 8, 0);
      compute();
    }
  } else {
    Regs g;
    const int nmax = nin > nd ? nin : nd;
    for (int row = r0 + w; row < r1; row += 4) {
      for (int base = 0; base < nmax; base += 256) { load(g, row, base); store(g, base, row); }
      compute();
    }
  }

  // ---- sum the four waves' tiles in fixed order, store the group slab ----
  float* red = sm;                                   // [4 waves][16 r][64 lanes]
  float* slab = a.part + (size_t)g * COUT * a.NP + (size_t)cb * 32 * a.NP;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(w * 16 + r) * 64 + lane] = acc[t][r];
    __syncthreads();
    const int nbase = (ky * KS + t / NCB) * CIN + (t % NCB) * 32;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = w + 4 * j;                       // element (r, lane) of the tile
      const int e = r * 64 + lane;
      const float v = (red[e] + red[1024 + e]) + (red[2048 + e] + red[3072 + e]);
      const int co = (r & 3) + 8 * (r >> 2) + 4 * h;
      slab[(size_t)co * a.NP + nbase + l31] = v;
    }
  }
  if (ky == 0) {   // bias column n = KC: lanes l, l+8, ... of every wave share channels
    __syncthreads();
    reinterpret_cast<float4*>(red)[w * 64 + lane] = bsum;
    __syncthreads();
    if (threadIdx.x < 32) {
      const int co = threadIdx.x, q = co >> 2, c = co & 3;
      float v = 0.f;
      for (int ww = 0; ww < 4; ++ww)
        for (int l = q; l < 64; l += 8) v += red[(ww * 64 + l) * 4 + c];
      slab[(size_t)co * a.NP + KC] = v;
    }
  }
}

template <int CIN, int COUT, int KS, int PAD, bool PSRC = false, int WPE = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void wgradd_kernel(
    const WgradDArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  wgradd_body<CIN, COUT, KS, PAD, PSRC>(a, sm, blockIdx.x);
}

template <int CIN, int PAD>
inline size_t wgradd_smem_bytes(int W) {
  const int f = 4 * WgradDGeom<CIN, PAD>::region(W);
  return (size_t)(f > 4096 ? f : 4096) * 4;
}

// Row groups: about two 4-wave workgroups per CU over all (cb, ky) pairs.
inline void wgradd_groups(int rows, int nts, int* G, int* RPG, int target = 512) {
  int g = target / nts;
  if (g >= 16) g &= ~7;            // whole XCD rounds (see the kernel's decode)
  if (g < 1) g = 1;
  if (g > rows) g = rows;
  const int rpg = (rows + g - 1) / g;
  *RPG = rpg;
  *G = (rows + rpg - 1) / rpg;
}

template <int CIN, int COUT, int KS, int PAD, bool PSRC = false, int WPE = 2>
inline hipError_t launch_wgradd(const WgradDArgs& a, hipStream_t st) {
  const size_t shm = wgradd_smem_bytes<CIN, PAD>(a.W);
  const int g8 = (a.G + 7) / 8 * 8;
  hipLaunchKernelGGL((wgradd_kernel<CIN, COUT, KS, PAD, PSRC, WPE>), dim3(g8 * (COUT / 32) * KS),
                     dim3(256), shm, st, a);
  return hipGetLastError();
}

}  // namespace ddq
