// Direct (patch-in-LDS) convolution kernels for the deepq conv layers (gfx950).
//
// One workgroup = one image b x one TY x TX tile of output pixels x all N
// output channels.  The input halo patch (TY+KS-1) x (TX+KS-1) x CP is staged
// in LDS ONCE (the implicit-GEMM path re-reads it KS^2 times through L1/L2),
// the weights tap by tap (two-slot ring, one barrier per tap) or all at once
// (WALL, conv1: 25 KB).  The MFMA operands are read straight from those
// images: for v_mfma_f32_32x32x2_f32 lane l = (row l&31, k-half h = l>>5)
// needs A[row][k] and B[k][col]; here each lane reads V = 4 (ds_read_b128) or
// V = 2 (ds_read_b64) consecutive channels per image and feeds V consecutive
// MFMA k-steps from them (half h owns channels [g*2V + h*V, +V) of group g),
// so there is no im2col, no per-element address arithmetic in the K loop and
// one LDS read per 4 MFMAs per operand block.
//
// WK > 1 splits the taps over WK wave groups (group g takes taps g, g+WK, ...,
// each with its own two-slot weight ring) and sums the groups' accumulators
// through LDS in fixed order before the epilogue: for layers whose output has
// too few 32x32 blocks to give every SIMD two waves (conv3: 512 per tower,
// conv2 dgrad: 1024) this multiplies the waves in flight by WK.
//
// Modes (template DGRAD):
//  fwd   : patch = layer input (CP channels), N = Cout, weights Wk[co][tap][ci];
//          epilogue = bias + ReLU + 2x2 max-pool + routing byte (rows are
//          window-major: a lane's 4 consecutive accumulator rows are one window).
//  dgrad : patch = this layer's dconv (CP = Cout channels), N = Cin, weights
//          transposed and tap-flipped while staged (conv with the flipped kernel,
//          pad KS-1-PAD); epilogue = un-pool + ReLU routing into the previous
//          layer's pre-pool gradient.  (Staging from a pre-transposed copy
//          kept by the apply kernel measured slower: 51.9 vs 40.4 us.)
#pragma once
#include <type_traits>

#include "common.h"
#include "split.h"

namespace ddq {

template <int CP, int N, int KS, int TY, int TX, int WM, int WN, bool DGRAD, bool WALL, int WK = 1,
          bool RB = false>
struct DirectCfg {
  static constexpr int V = CP >= 8 ? 4 : CP / 2;     // floats per lane per LDS read
  static constexpr int G = 2 * V;                     // channels per read group
  static constexpr int CS = CP >= 8 ? CP + 4 : CP;    // patch pixel stride (floats)
  static constexpr int PH = TY + KS - 1, PW = TX + KS - 1;
  // Patch row stride.  ds_read_b128 serves a wave in four 16-lane groups
  // (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) on 64 banks; a group
  // spans two pixel rows of the window-major block, so RS = 32 (mod 64)
  // puts the two rows in opposite bank halves: conflict-free (RS = 16 mod
  // 64 was 2-way, conv3's 40 mod 64 3-way).  CP < 8 (ds_read_b64, 32-lane
  // groups) is conflict-free at PW*CP + 2.
  static constexpr int RS0 = PW * CS + (CP >= 8 ? 0 : 2);
  static constexpr int RS = CP >= 8 ? RS0 + (96 - RS0 % 64) % 64 : RS0;
  // weight row stride (one row per n).  CP = 4 keeps stride 4 (2-way on the
  // ds_read_b64 B reads): stride 6 is conflict-free but its 37 KB weight
  // image costs conv1 a workgroup per CU (38.7 us against 30.7)
  static constexpr int CW = CP >= 8 ? CP + 4 : CP;
  static constexpr int T = KS * KS;
  static constexpr int WSLOTS = WALL ? T : 2 * WK;
  static constexpr int kGroup = 64 * WM * WN;         // threads of one tap group
  static constexpr int kThreads = kGroup * WK;
  static constexpr int TM = TY * TX / WM / 32;        // 32-pixel blocks per wave
  static constexpr int TN = N / WN / 32;              // 32-channel blocks per wave
  static constexpr int kPatch = PH * RS;
  static constexpr int kW = RB ? 0 : WSLOTS * N * CW;   // RB: weights never touch LDS
  static constexpr int kRed = (WK - 1) * WM * WN * TM * TN * 1024;   // tap-group sums
  static constexpr int kSmem = kPatch + kW > kRed ? kPatch + kW : kRed;
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  static_assert(TY % 2 == 0 && TX % 2 == 0 && CP % 4 == 0 && CP % G == 0, "shape");
  static_assert(kSmem * 4 <= 160 * 1024, "LDS budget");
};

struct DirectArgs {
  int B, H, W;               // conv grid (stride 1, same padding)
  int tiles_x;
  int pad;                   // spatial padding of the patch
  const float* in[2];        // patch source, NHWC (B,H,W,CP)
  const float* wk[2];        // Wk[co][tap][ci] of the layer
  const float* bias[2];      // fwd only
  float* out[2];             // fwd: pooled NHWC (B,H/2,W/2,N), or NCHW if nchw
  int nchw;                  // fwd: 1 = pooled output in Caffe (B,N,H/2,W/2) order
  int mask_nhwc;             // fwd, nchw: routing bytes stay NHWC (B,H/2,W/2,N)
  uint8_t* mask[2];          // fwd: routing bytes (nullable)
  // dgrad source given pooled: in = (B,H/2,W/2,CP) gradient of the pool
  // output, in_route = its NHWC routing bytes; the patch is staged as the
  // un-pooled gradient (value at the routed quadrant, 0 elsewhere)
  const uint8_t* in_route;
  const uint8_t* pmask;      // dgrad: previous pool's routing bytes (B,H,W,N)
  float* pdconv;             // dgrad: previous layer's pre-pool gradient (B,2H,2W,N)
  int pd_pooled;             // dgrad: 1 = store the pool-output gradient pooled, NHWC
                             // (B,H,W,N); the consumer routes it through pmask
  __bf16* pd_split;          // dgrad, pooled: also split (split.h), plane stride
  int64_t pd_split_elems;    // pd_split_elems (nullable)
};

template <int V>
struct VecT;
template <>
struct VecT<4> { using T = float4; };
template <>
struct VecT<2> { using T = float2; };

__device__ __forceinline__ float vget(const float4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}
__device__ __forceinline__ float vget(const float2& v, int i) { return i == 0 ? v.x : v.y; }

// Weight staging for one tap, split into a global->register load (issued
// before the previous tap's MFMAs) and a register->LDS store (after them).
template <class C, int CP, int N>
struct WStage {
  static constexpr int kF4 = N * CP / 4;                       // float4 per tap
  static constexpr int kPer = (kF4 + C::kGroup - 1) / C::kGroup;   // one tap group stages a tap
  static_assert(kPer <= 8, "weight staging slots");
  // Eight NAMED registers, every access through a compile-time slot: with a
  // float4 array member hipcc kept the staging set in scratch memory (48 B /
  // lane on conv2 fwd, seen in the .s), so the next tap's weight loads were
  // spilled the moment they landed instead of staying in flight.
  float4 r0, r1, r2, r3, r4, r5, r6, r7;

  template <int S>
  __device__ __forceinline__ float4& slot() {
    if constexpr (S == 0) return r0;
    else if constexpr (S == 1) return r1;
    else if constexpr (S == 2) return r2;
    else if constexpr (S == 3) return r3;
    else if constexpr (S == 4) return r4;
    else if constexpr (S == 5) return r5;
    else if constexpr (S == 6) return r6;
    else return r7;
  }
  template <int S>
  __device__ __forceinline__ const float4& slot() const {
    if constexpr (S == 0) return r0;
    else if constexpr (S == 1) return r1;
    else if constexpr (S == 2) return r2;
    else if constexpr (S == 3) return r3;
    else if constexpr (S == 4) return r4;
    else if constexpr (S == 5) return r5;
    else if constexpr (S == 6) return r6;
    else return r7;
  }

  // fwd: wb[n=co][k=ci] = Wk[co][t][ci], float4 along k.  dgrad (TRANS):
  // wb[n=ci][k=co] = Wk[co][T-1-t][ci], float4 along ci, transposed on store.
  template <bool TRANS, int S>
  __device__ __forceinline__ void load1(const float* __restrict__ wk, int t, int tid) {
    if constexpr (S < kPer) {
      const int f = tid + S * C::kGroup;
      if (kF4 % C::kGroup != 0 && f >= kF4) return;
      if (!TRANS) {
        const int n = f / (CP / 4), c4 = f % (CP / 4);
        slot<S>() = *reinterpret_cast<const float4*>(wk + ((size_t)n * C::T + t) * CP + 4 * c4);
      } else {
        const int co = f / (N / 4), n4 = f % (N / 4);
        slot<S>() = *reinterpret_cast<const float4*>(
            wk + ((size_t)co * C::T + (C::T - 1 - t)) * N + 4 * n4);
      }
    }
  }
  template <bool TRANS, int S>
  __device__ __forceinline__ void store1(float* wb, int tid) const {
    if constexpr (S < kPer) {
      const int f = tid + S * C::kGroup;
      if (kF4 % C::kGroup != 0 && f >= kF4) return;
      const float4 v = slot<S>();
      if (!TRANS) {
        const int n = f / (CP / 4), c4 = f % (CP / 4);
        *reinterpret_cast<float4*>(wb + n * C::CW + 4 * c4) = v;
      } else {
        const int co = f / (N / 4), n4 = f % (N / 4);
        wb[(4 * n4 + 0) * C::CW + co] = v.x;
        wb[(4 * n4 + 1) * C::CW + co] = v.y;
        wb[(4 * n4 + 2) * C::CW + co] = v.z;
        wb[(4 * n4 + 3) * C::CW + co] = v.w;
      }
    }
  }
  template <bool TRANS>
  __device__ __forceinline__ void load(const float* __restrict__ wk, int t, int tid) {
    load1<TRANS, 0>(wk, t, tid); load1<TRANS, 1>(wk, t, tid);
    load1<TRANS, 2>(wk, t, tid); load1<TRANS, 3>(wk, t, tid);
    load1<TRANS, 4>(wk, t, tid); load1<TRANS, 5>(wk, t, tid);
    load1<TRANS, 6>(wk, t, tid); load1<TRANS, 7>(wk, t, tid);
  }
  template <bool TRANS>
  __device__ __forceinline__ void store(float* wb, int tid) const {
    store1<TRANS, 0>(wb, tid); store1<TRANS, 1>(wb, tid);
    store1<TRANS, 2>(wb, tid); store1<TRANS, 3>(wb, tid);
    store1<TRANS, 4>(wb, tid); store1<TRANS, 5>(wb, tid);
    store1<TRANS, 6>(wb, tid); store1<TRANS, 7>(wb, tid);
  }
};

struct NoStage {
  template <bool TRANS>
  __device__ __forceinline__ void load(const float*, int, int) {}
  template <bool TRANS>
  __device__ __forceinline__ void store(float*, int) const {}
};

template <int CP, int N, int KS, int TY, int TX, int WM, int WN, bool DGRAD, bool WALL, int WK,
          bool RB>
__device__ __forceinline__ void direct_conv_body(const DirectArgs& a, float* smem, int bx, int by,
                                                 int bz) {
  using C = DirectCfg<CP, N, KS, TY, TX, WM, WN, DGRAD, WALL, WK, RB>;
  static_assert(!(RB && WALL), "register-B is per-tap");
  using VT = typename VecT<C::V>::T;
  constexpr int TM = C::TM, TN = C::TN, V = C::V;
  float* patch = smem;
  float* wbuf = smem + C::kPatch;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wkg = wid / (WM * WN);                 // tap group: taps t = s*WK + wkg
  const int gtid = tid - wkg * C::kGroup;
  const int z = bz, b = by;
  const int ty = bx / a.tiles_x, tx = bx % a.tiles_x;
  const int y0 = ty * TY, x0 = tx * TX;
  // select, never index, the per-tower kernel arguments: a runtime index into
  // a kernarg array makes the compiler copy the struct to scratch memory
  const float* __restrict__ in = z ? a.in[1] : a.in[0];
  const float* __restrict__ wk = z ? a.wk[1] : a.wk[0];
  const float* __restrict__ biasz = z ? a.bias[1] : a.bias[0];
  float* __restrict__ outz = z ? a.out[1] : a.out[0];
  uint8_t* __restrict__ maskz = z ? a.mask[1] : a.mask[0];

  // ---- stage the halo patch (zero outside the image) and the first weights ----
  // (register-B kernels never stage weights: a stand-in keeps the code shared)
  std::conditional_t<RB, NoStage, WStage<C, CP, N>> ws;
  if constexpr (WALL) {
    // every global load (patch, and the weights: all taps for WALL, the
    // group's first tap otherwise) is issued before the first LDS store, so
    // the prologue pays one memory latency instead of one per staging round
    // (conv1: -12 us in the kernel trace)
    constexpr int kPF4 = C::PH * C::PW * (CP / 4);
    constexpr int kPIt = (kPF4 + C::kThreads - 1) / C::kThreads;
    constexpr int kWF4 = WALL ? C::T * N * (CP / 4) : 1;
    constexpr int kWIt = (kWF4 + C::kThreads - 1) / C::kThreads;
    static_assert(!(WALL && DGRAD), "WALL staging is forward-only");
    float4 pv[kPIt], wv[kWIt];
#pragma unroll
    for (int it = 0; it < kPIt; ++it) {
      const int f = tid + it * C::kThreads;
      pv[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kPF4 % C::kThreads == 0 || f < kPF4) {
        const int pix = f / (CP / 4), c4 = f % (CP / 4);
        const int py = pix / C::PW, px = pix % C::PW;
        const int gy = y0 - a.pad + py, gx = x0 - a.pad + px;
        if ((unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W)
          pv[it] = *reinterpret_cast<const float4*>(in + (((size_t)b * a.H + gy) * a.W + gx) * CP +
                                                     4 * c4);
      }
    }
    if constexpr (WALL) {
#pragma unroll
      for (int it = 0; it < kWIt; ++it) {
        const int f = tid + it * C::kThreads;
        wv[it] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kWF4 % C::kThreads == 0 || f < kWF4) wv[it] = reinterpret_cast<const float4*>(wk)[f];
      }
    } else {
      if (wkg < C::T) ws.template load<DGRAD>(wk, wkg, gtid);
    }
#pragma unroll
    for (int it = 0; it < kPIt; ++it) {
      const int f = tid + it * C::kThreads;
      if (kPF4 % C::kThreads == 0 || f < kPF4) {
        const int pix = f / (CP / 4), c4 = f % (CP / 4);
        const int py = pix / C::PW, px = pix % C::PW;
        float* dst = patch + py * C::RS + px * C::CS + 4 * c4;
        if (CP >= 8) {
          *reinterpret_cast<float4*>(dst) = pv[it];
        } else {
          reinterpret_cast<float2*>(dst)[0] = make_float2(pv[it].x, pv[it].y);
          reinterpret_cast<float2*>(dst)[1] = make_float2(pv[it].z, pv[it].w);
        }
      }
    }
    if constexpr (WALL) {
#pragma unroll
      for (int it = 0; it < kWIt; ++it) {
        const int f = tid + it * C::kThreads;
        if (kWF4 % C::kThreads == 0 || f < kWF4) {
          const int n = f / (C::T * (CP / 4)), rem = f % (C::T * (CP / 4));
          const int t = rem / (CP / 4), c4 = rem % (CP / 4);
          float* dst = wbuf + (t * N + n) * C::CW + 4 * c4;
          if (CP >= 8) {
            *reinterpret_cast<float4*>(dst) = wv[it];
          } else {
            reinterpret_cast<float2*>(dst)[0] = make_float2(wv[it].x, wv[it].y);
            reinterpret_cast<float2*>(dst)[1] = make_float2(wv[it].z, wv[it].w);
          }
        }
      }
    } else {
      if (wkg < C::T) ws.template store<DGRAD>(wbuf + wkg * N * C::CW, gtid);
    }
  } else {
    for (int f = tid; f < C::PH * C::PW * (CP / 4); f += C::kThreads) {
      const int pix = f / (CP / 4), c4 = f % (CP / 4);
      const int py = pix / C::PW, px = pix % C::PW;
      const int gy = y0 - a.pad + py, gx = x0 - a.pad + px;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W) {
        if (DGRAD && a.in_route) {   // pooled source: expand through the routing bytes
          const size_t o =
              (((size_t)b * (a.H >> 1) + (gy >> 1)) * (a.W >> 1) + (gx >> 1)) * CP + 4 * c4;
          const float4 u = *reinterpret_cast<const float4*>(in + o);
          const uint32_t m = *reinterpret_cast<const uint32_t*>(a.in_route + o);
          const uint32_t q = ((gy & 1) << 1) | (gx & 1);
          v.x = (m & 0xff) == q ? u.x : 0.f;
          v.y = ((m >> 8) & 0xff) == q ? u.y : 0.f;
          v.z = ((m >> 16) & 0xff) == q ? u.z : 0.f;
          v.w = (m >> 24) == q ? u.w : 0.f;
        } else {
          v = *reinterpret_cast<const float4*>(in + (((size_t)b * a.H + gy) * a.W + gx) * CP +
                                               4 * c4);
        }
      }
      float* dst = patch + py * C::RS + px * C::CS + 4 * c4;
      if (CP >= 8) {
        *reinterpret_cast<float4*>(dst) = v;
      } else {
        reinterpret_cast<float2*>(dst)[0] = make_float2(v.x, v.y);
        reinterpret_cast<float2*>(dst)[1] = make_float2(v.z, v.w);
      }
    }
    if (!RB && wkg < C::T) {
      ws.template load<DGRAD>(wk, wkg, gtid);
      ws.template store<DGRAD>(wbuf + wkg * N * C::CW, gtid);
    }
  }
  __syncthreads();

  // ---- per-lane operand bases ----
  const int l31 = lane & 31, h = lane >> 5;
  const int w2 = wid % (WM * WN);
  const int wmi = w2 / WN, wni = w2 % WN;
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wmi * TM * 32 + 32 * i + l31;
    const int win = m >> 2, dy = (m >> 1) & 1, dx = m & 1;
    const int wy = win / (TX / 2), wx = win % (TX / 2);
    abase[i] = (2 * wy + dy) * C::RS + (2 * wx + dx) * C::CS + h * V;
  }
  int bbase[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bbase[j] = (wni * TN * 32 + 32 * j + l31) * C::CW + h * V;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Tap steps: group wkg takes tap s*WK + wkg; non-WALL weights live in a
  // two-slot ring per group (slot (s&1)*WK + wkg), one barrier per step.
  constexpr int NSTEP = (C::T + WK - 1) / WK;
  if constexpr (RB) {
    // Register-B: every lane loads its own B operand of the next tap straight
    // from the (L2-resident) weights while this tap's MFMAs run -- no weight
    // staging, no LDS weight reads, no barrier in the tap loop, and LDS holds
    // only the patch (more workgroups per CU).
    //   fwd  : B[k = ci][n = co] = Wk[co][t][ci]      (one VT load per group)
    //   dgrad: B[k = co][n = ci] = Wk[co][T-1-t][ci]  (V dword loads, lanes
    //          along ci: 128-byte rows)
    constexpr int NG = CP / C::G;
    float bq[2][TN][NG][V];
    auto load_b = [&](float (&dst)[TN][NG][V], int t) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wni * TN * 32 + 32 * j + l31;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          const int k0 = g * C::G + h * V;
          if (!DGRAD) {
            const VT q = *reinterpret_cast<const VT*>(wk + ((size_t)n * C::T + t) * CP + k0);
#pragma unroll
            for (int v = 0; v < V; ++v) dst[j][g][v] = vget(q, v);
          } else {
#pragma unroll
            for (int v = 0; v < V; ++v)
              dst[j][g][v] = wk[((size_t)(k0 + v) * C::T + (C::T - 1 - t)) * N + n];
          }
        }
      }
    };
    load_b(bq[0], wkg < C::T ? wkg : C::T - 1);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      const int t = s * WK + wkg;
      const int tn = t + WK;
      if (s + 1 < NSTEP) load_b(bq[(s + 1) & 1], tn < C::T ? tn : C::T - 1);
      __builtin_amdgcn_sched_barrier(0);
      if (t < C::T) {
        const int ky = t / KS, kx = t % KS;
        const float* pa = patch + ky * C::RS + kx * C::CS;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          VT av[TM];
#pragma unroll
          for (int i = 0; i < TM; ++i)
            av[i] = *reinterpret_cast<const VT*>(pa + abase[i] + g * C::G);
#pragma unroll
          for (int v = 0; v < V; ++v)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                    vget(av[i], v), bq[s & 1][j][g][v], acc[i][j], 0, 0, 0);
        }
      }
    }
  } else
  for (int s = 0; s < NSTEP; ++s) {
    const int t = s * WK + wkg;
    const int tn = t + WK;
    const float* wb = wbuf + (WALL ? t : ((s & 1) * WK + wkg)) * N * C::CW;
    // next tap's weights in flight under this tap's MFMAs (clamped index: the
    // load is unconditional so the staging registers never go through scratch)
    if (!WALL && s + 1 < NSTEP) {
      ws.template load<DGRAD>(wk, tn < C::T ? tn : C::T - 1, gtid);
      // pin the loads here: without the barrier hipcc sinks them to the LDS
      // store after the MFMAs and waits on them at once (one exposed L2
      // round trip per tap, seen in the .s)
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t < C::T) {
      const int ky = t / KS, kx = t % KS;
      const float* pa = patch + ky * C::RS + kx * C::CS;
#pragma unroll
      for (int g = 0; g < CP / C::G; ++g) {
        VT av[TM], bv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) av[i] = *reinterpret_cast<const VT*>(pa + abase[i] + g * C::G);
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = *reinterpret_cast<const VT*>(wb + bbase[j] + g * C::G);
#pragma unroll
        for (int v = 0; v < V; ++v)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vget(av[i], v), vget(bv[j], v),
                                                               acc[i][j], 0, 0, 0);
      }
    }
    if (!WALL && s + 1 < NSTEP) {
      // the other slot was last read in step s-1, fenced by its barrier
      if (tn < C::T) ws.template store<DGRAD>(wbuf + (((s + 1) & 1) * WK + wkg) * N * C::CW, gtid);
      __syncthreads();
    }
  }

  // ---- tap groups 1..WK-1 hand their partial sums to group 0 (fixed order) ----
  if (WK > 1) {
    __syncthreads();
    float* red = smem;
    if (wkg > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            red[((((wkg - 1) * WM * WN + w2) * TM + i) * TN + j) * 1024 + r * 64 + lane] =
                acc[i][j][r];
    }
    __syncthreads();
    if (wkg > 0) return;
#pragma unroll
    for (int k = 1; k < WK; ++k)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            acc[i][j][r] += red[((((k - 1) * WM * WN + w2) * TM + i) * TN + j) * 1024 + r * 64 + lane];
  }

  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int mb = wmi * TM * 32 + 32 * i;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wni * TN * 32 + 32 * j + l31;
      if (!DGRAD) {
        const int Hp = a.H >> 1, Wp = a.W >> 1;
        const float bv = biasz[n];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int win = (mb + 8 * g + 4 * h) >> 2;
          const int pyy = y0 / 2 + win / (TX / 2), pxx = x0 / 2 + win % (TX / 2);
          if (pyy >= Hp || pxx >= Wp) continue;
          float v0 = acc[i][j][4 * g + 0] + bv, v1 = acc[i][j][4 * g + 1] + bv;
          float v2 = acc[i][j][4 * g + 2] + bv, v3 = acc[i][j][4 * g + 3] + bv;
          float mx = v0; int arg = 0;
          if (v1 > mx) { mx = v1; arg = 1; }
          if (v2 > mx) { mx = v2; arg = 2; }
          if (v3 > mx) { mx = v3; arg = 3; }
          const bool pos = mx > 0.f;
          const size_t onhwc = (((size_t)b * Hp + pyy) * Wp + pxx) * N + n;
          const size_t o = a.nchw ? (((size_t)b * N + n) * Hp + pyy) * Wp + pxx : onhwc;
          outz[o] = pos ? mx : 0.f;
          if (maskz) maskz[a.mask_nhwc ? onhwc : o] = (uint8_t)(pos ? arg : 4);
        }
      } else {
        const int W2 = 2 * a.W;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mb + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int win = m >> 2;
          const int y = y0 + 2 * (win / (TX / 2)) + ((m >> 1) & 1);
          const int x = x0 + 2 * (win % (TX / 2)) + (m & 1);
          if (y >= a.H || x >= a.W) continue;
          const size_t pix = ((size_t)b * a.H + y) * a.W + x;
          const float v = acc[i][j][r];
          if (a.pd_pooled) {   // one store per element: lanes along n, 128-B runs
            if (a.pdconv) a.pdconv[pix * N + n] = v;   // null: split copy only
            if (a.pd_split)   // written through (split.h wt_store_split)
              wt_store_split(wt_rsrc(a.pd_split, (uint32_t)a.pd_split_elems * 6),
                             (uint32_t)a.pd_split_elems, (uint32_t)(pix * N + n), v);
            continue;
          }
          const int mk = a.pmask[pix * N + n];
          float* base = a.pdconv + (((size_t)b * 2 * a.H + 2 * y) * W2 + 2 * x) * N + n;
          base[0] = (mk == 0) ? v : 0.f;
          base[N] = (mk == 1) ? v : 0.f;
          base[(size_t)W2 * N] = (mk == 2) ? v : 0.f;
          base[(size_t)W2 * N + N] = (mk == 3) ? v : 0.f;
        }
      }
    }
  }
}

template <int CP, int N, int KS, int TY, int TX, int WM, int WN, bool DGRAD, bool WALL, int WK,
          bool RB>
__global__ __launch_bounds__(64 * WM * WN * WK) void direct_conv_kernel(const DirectArgs a) {
  using C = DirectCfg<CP, N, KS, TY, TX, WM, WN, DGRAD, WALL, WK, RB>;
  __shared__ __attribute__((aligned(16))) float smem[C::kSmem];
  direct_conv_body<CP, N, KS, TY, TX, WM, WN, DGRAD, WALL, WK, RB>(a, smem, blockIdx.x, blockIdx.y,
                                                                  blockIdx.z);
}

template <int CP, int N, int KS, int TY, int TX, int WM, int WN, bool DGRAD, bool WALL, int WK = 1,
          bool RB = false>
inline hipError_t launch_direct(DirectArgs a, int nz, hipStream_t st) {
  a.tiles_x = (a.W + TX - 1) / TX;
  const int tiles_y = (a.H + TY - 1) / TY;
  dim3 grid(tiles_y * a.tiles_x, a.B, nz);
  hipLaunchKernelGGL((direct_conv_kernel<CP, N, KS, TY, TX, WM, WN, DGRAD, WALL, WK, RB>), grid,
                     dim3(64 * WM * WN * WK), 0, st, a);
  return hipGetLastError();
}

}  // namespace ddq
