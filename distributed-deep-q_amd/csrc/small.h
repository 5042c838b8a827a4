// The deepq16 step (S = 16, train_val.prototxt:8-11) in four launches.
//
// At 16 x 16 every layer of the 64 x 64 path is one tile per image: eleven
// launches of 4-17 us each, bound by their launch and by the weights each
// workgroup streams from L2 with two steps of lookahead (conv2 forward: 307
// KB of split weights per workgroup behind 25 dependent ring steps), not by
// MFMA work (the whole step is 1.4 GFLOP).  Here:
//
//   K1 tower_fwd16   one workgroup per (image, tower): conv1 -> pool1 ->
//                    conv2 -> pool2 -> conv3 -> pool3 with the activations in
//                    LDS (split bf16 planes, zero halos), the weights through
//                    a two-slot LDS ring fed K taps ahead from registers, the
//                    next layer's first taps issued under the current one.
//                    Writes pool3 (fc4's input), the Q tower's routing bytes
//                    and its split pool1 / pool2 (the weight gradients').
//   K2 fc4_chain16   fc4 forward, head and fc4 backward (small.h part 2)
//   K3 tower_bwd16   conv3 / conv2 data gradients per image, conv1's weight
//                    gradient slab (part 3)
//   K4 wgrad16       conv2 / conv3 weight gradients, slab sums, apply (part 4)
//
// Arithmetic is the 64 x 64 path's (split.h): split bf16 operands, six MFMA
// products into an fp32 accumulator pair (three for conv1's exact frames).
#pragma once
#include "kernels.h"
#include "split.h"

namespace ddq {
namespace sm16 {

constexpr int kS = 16;
constexpr int kThreads = 512;
// conv1 patch (split.h Conv1Cfg<16, 16, 8>): 22 rows x 24 pixels x 4 ch
constexpr int C1_PH = 22, C1_PW = 24, C1_RS = 192, C1_CW = 232;
// conv2 input image: pool1 8 x 8 x 32 with a zero halo of 2 -> 12 x 12 pixels,
// pixel stride 40 bf16 (an odd number of 16-byte units), row stride == 64
// (mod 128) bf16 (split.h SplitCfg, MF 0)
constexpr int P1_CS = 40, P1_RS = 576, P1_PL = 12 * P1_RS;
constexpr int W2_CW = 40, W2_PL = 64 * W2_CW, W2_SLOT = 3 * W2_PL;      // bf16
// conv3 input image: pool2 4 x 4 x 64, halo 1 -> 6 x 6, pixel stride 80 (MF 1)
constexpr int P2_CS = 80, P2_RS = 576, P2_PL = 6 * P2_RS;
constexpr int W3_CW = 80, W3_PL = 64 * W3_CW, W3_SLOT = 3 * W3_PL;      // bf16
// LDS map (bytes).  P1 / P2 / the routing bytes live all kernel long (the
// global outputs are written from them at the end, so no load wait of the
// weight pipeline ever waits on a store); region R is conv1's patch and
// weights, then conv2's ring, the k-half sums, then conv3's ring.
constexpr int OFF_P1 = 0;                                  // 41472
constexpr int OFF_P2 = 41472;                              // 20736
constexpr int OFF_STG1 = 62208;                            // pool1 routing bytes 2048
constexpr int OFF_STG2 = 64256;                            // pool2 routing bytes 1024
constexpr int OFF_R = 65280;
constexpr int OFF_PATCH = OFF_R;                           // conv1 patch 8448
constexpr int OFF_W1 = OFF_PATCH + C1_PH * C1_RS * 2;      // conv1 weights 44544
constexpr int OFF_RING2 = OFF_R;                           // 3 x 15360
constexpr int OFF_RED = OFF_R;                             // 4 waves x 16 x 64 fp32
constexpr int OFF_RING3 = OFF_R;                           // 3 x 30720
constexpr int kFwdSmem = OFF_RING3 + 3 * W3_SLOT * 2;      // 157440
static_assert(3 * P1_PL * 2 == 41472 && 3 * P2_PL * 2 == 20736, "image sizes");
static_assert(OFF_W1 + 3 * 32 * C1_CW * 2 <= kFwdSmem, "conv1 region");
static_assert(kFwdSmem <= 160 * 1024, "LDS");

// the fused apply's bookkeeping and the next step's draw (launch_head's
// latch / bump / head_draw), run by one extra workgroup of K1
struct BookArgs {
  int32_t* latch;              // opt_init: [2] first call, [3] P <- Q sync due (nullable)
  const int64_t* iter;
  int period, inc;
  ReplayMeta* bump;            // counter += 1 (nullable)
  ReplayMeta* dmeta;           // or: draw the next step's set with counter + 1 (nullable)
  int32_t* didx;
  uint64_t dseed;
  int32_t* dlog;
  int64_t dlog_cap;
  int B;
};

struct TowerArgs {
  int B, nz;
  const float* in[2];          // frames, fp32 NHWC (B, 16, 16, 4): exact integers
  const __bf16* wks[2];        // split forward weights (split.h; plane stride wks_plane)
  int64_t wks_plane, wks_off2, wks_off3;
  const float* bias1[2];
  const float* bias2[2];
  const float* bias3[2];
  __bf16* pool1s;              // Q: split pool1 NHWC (B, 8, 8, 32), plane stride B*2048
  __bf16* pool2s;              // Q: split pool2 NHWC (B, 4, 4, 64), plane stride B*1024
  uint8_t *mask1, *mask2, *mask3;   // Q: NHWC routing bytes (0..3 first max, 4 ReLU'd)
  float* pool3[2];             // Caffe (B, 64, 2, 2)
  BookArgs bk;
  // the data gradients' transposed split weights of Q (K3 reads them), made
  // from wks[0] by ntr extra workgroups (25 conv2 taps, 9 conv3 taps)
  int ntr;
  int64_t wks2_off, wkst_off, wks3_off, wkst3_off;
  // split form (tower_fwd16s): the pool2 halves' exchange
  __bf16* xchg;                // [B][nz][2 halves][3 planes][16 px][32 ch]
  uint64_t* pairc;             // [B][nz] meeting counters
  int32_t* timeout;            // sticky spin timeout
};

// pool of a 2x2 window (v0..v3 in window order: (0,0) (0,1) (1,0) (1,1)),
// bias, ReLU; first-max routing byte, 4 = ReLU'd window (split.h epilogue)
__device__ __forceinline__ float pool4(float v0, float v1, float v2, float v3, float bias,
                                       uint8_t& route) {
  v0 += bias; v1 += bias; v2 += bias; v3 += bias;
  float mx = v0;
  int arg = 0;
  if (v1 > mx) { mx = v1; arg = 1; }
  if (v2 > mx) { mx = v2; arg = 2; }
  if (v3 > mx) { mx = v3; arg = 3; }
  const bool pos = mx > 0.f;
  route = (uint8_t)(pos ? arg : 4);
  return pos ? mx : 0.f;
}

__device__ __forceinline__ void lds_split3(__bf16* p, int plane, float v) {
  __bf16 h, m, l;
  split3(v, h, m, l);
  p[0] = h;
  p[plane] = m;
  p[2 * plane] = l;
}

// conv2 weight taps: 3 planes x 64 co x 32 ci = 768 16-byte vectors, thread f
// and f + 512 (f < 256).  Rows n and n + 4 share an 8-lane ds_write group
// (SplitWStage::row): conflict-free stores of the 40-bf16 rows.
struct W2Tap {
  u32x4 r[2];
  static __device__ __forceinline__ void coords(int f, int& p, int& n, int& c8) {
    p = f >> 8;
    const int q = f & 255, n0 = q >> 2;
    c8 = q & 3;
    n = (n0 & ~7) | ((n0 & 7) >> 1) | ((n0 & 1) << 2);
  }
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int tap,
                                       int tid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int f = s ? (tid < 256 ? tid + 512 : tid) : tid;   // the second: 256 live
      int p, n, c8;
      coords(f, p, n, c8);
      r[s] = *reinterpret_cast<const u32x4*>(wk + p * plane + (n * 25 + tap) * 32 + 8 * c8);
    }
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s && tid >= 256) continue;
      const int f = tid + 512 * s;
      int p, n, c8;
      coords(f, p, n, c8);
      *reinterpret_cast<u32x4*>(slot + p * W2_PL + n * W2_CW + 8 * c8) = r[s];
    }
  }
};

// conv3 weight taps: 3 planes x 64 co x 64 ci = 1536 vectors, 3 per thread
// (plane s: row tid / 8, 16-byte column tid % 8: whole 128-byte row segments)
struct W3Tap {
  u32x4 r[3];
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int tap,
                                       int tid) {
    const int n = tid >> 3, c8 = tid & 7;
#pragma unroll
    for (int s = 0; s < 3; ++s)
      r[s] = *reinterpret_cast<const u32x4*>(wk + s * plane + (n * 9 + tap) * 64 + 8 * c8);
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
    const int n = tid >> 3, c8 = tid & 7;
#pragma unroll
    for (int s = 0; s < 3; ++s)
      *reinterpret_cast<u32x4*>(slot + s * W3_PL + n * W3_CW + 8 * c8) = r[s];
  }
};

__device__ void book_block(const BookArgs& k);
__device__ void tower_transpose(const TowerArgs& a, int x, char* smem);

// n workgroups meet: returns in each once all n have arrived (their stores
// write-through and drained: visible to sc1 loads, MI355X_MICROARCH.md
// inter-workgroup visibility, table row 1).  One monotonic 64-bit counter per
// meeting point, never reset: arrival `old` belongs to the group ending at
// (old / n + 1) n, which its last arriver reaches with its own add (no
// reset / generation round trips on the release path).  Bounded: a spin past
// ~0.1 s records a timeout in the sticky word and goes on (no hang); callers
// read the word afterwards (meet_failed) and then write no parameter.
__device__ __forceinline__ void meet(uint64_t* ctr, uint32_t n, int32_t* timeout) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t old = __hip_atomic_fetch_add(ctr, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t target = (old / n + 1) * n;
    if (old + 1 != target) {
      int spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 21)) {
          __hip_atomic_store(timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

// After a meet(): did this meeting (or an earlier one of the step) fail?  The
// sticky word is set by a party whose spin gave up before it left the
// meeting, and a party that arrives after the others gave up finds it set.
// One sc1 load (L2-served: the word is written by other workgroups of this
// launch), issued right after the meeting and consumed only where the
// parameters are written, so no path waits on it.
__device__ __forceinline__ int32_t meet_word(const int32_t* w) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(w), (short)0, 4, 0x00020000);
  return __builtin_bit_cast(int32_t, __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 16));
}

// An earlier launch of this step failed a meeting (its sticky timeout word,
// written before this launch began -- the kernel boundary made it visible,
// so plain loads): this launch writes no parameters.
__device__ __forceinline__ bool step_poisoned(const int32_t* w0, const int32_t* w1) {
  return (w0 && *w0 != 0) || (w1 && *w1 != 0);
}


// ---------------------------------------------------------------------------
// K1.  Waves: conv1 one 32-pixel block each (8 x 32 = 256 pixels,
// window-major); conv2 (m block, n block, k half) = 2 x 2 x 2 on 32x32x16;
// conv3 (n block, k step) = 4 x 2 on 16x16x32 (16 pixels x 16 channels).
// conv2 / conv3 run a three-slot weight ring: at tap t a wave issues the
// global loads of tap t + K (registers), reads tap t + 1's operands out of
// LDS (the MFMAs of tap t use the ones read at t - 1: no LDS latency between
// barrier and MFMA), issues tap t's MFMAs, stores tap t + 2 into the slot tap
// t - 1 used, and meets the others at one barrier.
// ---------------------------------------------------------------------------
template <int K2, int K3>
__global__ __launch_bounds__(kThreads) void tower_fwd16_kernel(const TowerArgs a) {
  static_assert(K2 >= 3 && K3 >= 3, "ring: tap t + 2 is stored from registers at tap t");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  if (bid >= a.B * a.nz) {
    if (bid - a.B * a.nz < a.ntr) tower_transpose(a, bid - a.B * a.nz, smem);
    else book_block(a.bk);
    return;
  }
  DDQ_STAMP(0);
  const int z = bid % a.nz, b = bid / a.nz;
  const bool q_tower = z == 0;
  const __bf16* __restrict__ wk1 = a.wks[z];
  const __bf16* __restrict__ wk2 = a.wks[z] + a.wks_off2;
  const __bf16* __restrict__ wk3 = a.wks[z] + a.wks_off3;
  const int64_t wpl = a.wks_plane;
  __bf16* P1 = reinterpret_cast<__bf16*>(smem + OFF_P1);
  __bf16* P2 = reinterpret_cast<__bf16*>(smem + OFF_P2);
  __bf16* patch = reinterpret_cast<__bf16*>(smem + OFF_PATCH);
  __bf16* w1s = reinterpret_cast<__bf16*>(smem + OFF_W1);
  __bf16* ring2 = reinterpret_cast<__bf16*>(smem + OFF_RING2);
  __bf16* ring3 = reinterpret_cast<__bf16*>(smem + OFF_RING3);
  float* red = reinterpret_cast<float*>(smem + OFF_RED);
  uint8_t* stg1 = reinterpret_cast<uint8_t*>(smem + OFF_STG1);
  uint8_t* stg2 = reinterpret_cast<uint8_t*>(smem + OFF_STG2);

  // ---- prologue: the frames' patch and conv1's weights first (conv1 waits
  // for them), then conv2's first K2 taps (they land under conv1) ----
  constexpr int NP = C1_PH * C1_PW;                 // 528 patch pixels
  float4 fv[2];
  {
    const float* __restrict__ in = a.in[z];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int f = tid + it * kThreads;
      const int py = f / C1_PW, px = f % C1_PW;
      const int gy = py - 3, gx = px - 3;
      fv[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < NP && px < kS + 6 && (unsigned)gy < (unsigned)kS && (unsigned)gx < (unsigned)kS)
        fv[it] = *reinterpret_cast<const float4*>(in + (((size_t)b * kS + gy) * kS + gx) * 4);
    }
  }
  constexpr int NW1 = 3 * kConv1WPlane / 8;         // 2688 vectors
  constexpr int WIT = (NW1 + kThreads - 1) / kThreads;
  u32x4 wv[WIT];
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int f0 = tid + it * kThreads;
    const int f = f0 < NW1 ? f0 : NW1 - 1;
    const int p = f / (kConv1WPlane / 8), r = f % (kConv1WPlane / 8);
    wv[it] = *reinterpret_cast<const u32x4*>(wk1 + p * wpl + 8 * (size_t)r);
  }
  const float bias1 = a.bias1[z][l31];
  const int wm2 = wid & 1, wn2 = (wid >> 1) & 1, wk2g = wid >> 2;
  const float bias2 = a.bias2[z][32 * wn2 + l31];
  const int wn3 = wid & 3, wk3g = wid >> 2;
  const float bias3 = a.bias3[z][16 * wn3 + (lane & 15)];
  W2Tap w2[K2];
#pragma unroll
  for (int k = 0; k < K2; ++k) w2[k].load(wk2, wpl, k, tid);
  // zero the two activation images (their halos must read 0)
  for (int f = tid; f < (3 * P1_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(P1)[f] = u32x4{0u, 0u, 0u, 0u};
  for (int f = tid; f < (3 * P2_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(P2)[f] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int f = tid + it * kThreads;
    if (f < NP) {
      const int py = f / C1_PW, px = f % C1_PW;
      __bf16 q[4] = {(__bf16)fv[it].x, (__bf16)fv[it].y, (__bf16)fv[it].z, (__bf16)fv[it].w};
      *reinterpret_cast<uint2*>(patch + py * C1_RS + px * 4) = *reinterpret_cast<uint2*>(q);
    }
  }
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int f0 = tid + it * kThreads;
    if (f0 < NW1) {
      const int p = f0 / (kConv1WPlane / 8), r = f0 % (kConv1WPlane / 8);
      const int n = r / 28, q8 = r % 28;
      *reinterpret_cast<u32x4*>(w1s + (p * 32 + n) * C1_CW + 8 * q8) = wv[it];
    }
  }
  __syncthreads();
  DDQ_STAMP(1);

  // ---- conv1: wave wid = pixels [32 wid, +32) window-major (split_conv1) ----
  {
    f32x16 acc, cor;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[r] = 0.f; cor[r] = 0.f; }
    const int m = wid * 32 + l31;
    const int win = m >> 2, dy = (m >> 1) & 1, dx = m & 1;
    const int wy = win >> 3, wx = win & 7;
    const int abase = (2 * wy + dy) * C1_RS + (2 * wx + dx + 2 * h) * 4;
    const int bbase = l31 * C1_CW + h * 8;
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        bf16x8 bv[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bv[p] = *reinterpret_cast<const bf16x8*>(w1s + p * 32 * C1_CW + bbase + ky * 32 + 16 * g);
        typedef __attribute__((address_space(3))) const u32x2 lds_u2;
        typedef __attribute__((address_space(3))) const char lds_c;
        lds_u2* la = (lds_u2*)(patch + abase + ky * C1_RS + 16 * g);
        uint32_t hi_off = 8;                        // opaque: two ds_read_b64 (split.h)
        asm volatile("" : "+v"(hi_off));
        const u32x2 lo = *la;
        const u32x2 hi = *(lds_u2*)((lds_c*)la + hi_off);
        u32x4 av4 = {lo[0], lo[1], hi[0], hi[1]};
        const bf16x8 av = *reinterpret_cast<bf16x8*>(&av4);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[2], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[1], cor, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[0], acc, 0, 0, 0);
      }
    }
    acc += cor;
    DDQ_STAMP(2);
    // epilogue: lane rows 8g + 4h + 0..3 = window 8 wid + 2g + h, channel l31;
    // the pooled value goes split into P1 at (py + 2, px + 2)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int wn = 8 * wid + 2 * g + h;           // pooled pixel (wn >> 3, wn & 7)
      uint8_t rt;
      const float o = pool4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3], bias1, rt);
      lds_split3(P1 + ((wn >> 3) + 2) * P1_RS + ((wn & 7) + 2) * P1_CS + l31, P1_PL, o);
      stg1[wn * 32 + l31] = rt;
    }
  }
  __syncthreads();   // P1 complete; conv1's patch / weights dead
  // conv2's taps 0 and 1 into ring slots 0 and 1 (over the dead conv1 region)
  w2[0].store(ring2, tid);
  w2[1].store(ring2 + W2_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(3);

  // ---- conv2: 25 taps ----
  W3Tap w3[K3];
  {
    f32x16 acc, cor;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[r] = 0.f; cor[r] = 0.f; }
    const int m = 32 * wm2 + l31;
    const int win = m >> 2, dy = (m >> 1) & 1, dx = m & 1;
    const int y = 2 * (win >> 2) + dy, x = 2 * (win & 3) + dx;
    const int abase = y * P1_RS + x * P1_CS + 16 * wk2g + 8 * h;
    const int bbase = (32 * wn2 + l31) * W2_CW + 16 * wk2g + 8 * h;
    bf16x8 av[2][3], bv[2][3];
    auto ops = [&](int t, int set) {
      const __bf16* wb = ring2 + (t % 3) * W2_SLOT;
      const __bf16* pa = P1 + (t / 5) * P1_RS + (t % 5) * P1_CS;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        av[set][p] = *reinterpret_cast<const bf16x8*>(pa + p * P1_PL + abase);
        bv[set][p] = *reinterpret_cast<const bf16x8*>(wb + p * W2_PL + bbase);
      }
    };
    ops(0, 0);
#pragma unroll
    for (int t = 0; t < 25; ++t) {
      if (t + K2 < 25) {
        w2[(t + K2) % K2].load(wk2, wpl, t + K2, tid);
      } else if (t + K2 - 25 < K3) {   // conv3's first taps under conv2's last ones
        w3[t + K2 - 25].load(wk3, wpl, t + K2 - 25, tid);
      }
      if (t + 1 < 25) ops(t + 1, (t + 1) & 1);
      const int c = t & 1;
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][2], bv[c][0], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][1], bv[c][1], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][0], bv[c][2], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][1], bv[c][0], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][0], bv[c][1], cor, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][0], bv[c][0], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < 25) w2[(t + 2) % K2].store(ring2 + ((t + 2) % 3) * W2_SLOT, tid);
      __syncthreads();
    }
    acc += cor;
    DDQ_STAMP(4);
    // k halves meet in LDS (fixed order: half 0 + half 1); half 0 finishes
    if (wk2g == 1) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wid & 3) * 16 + r) * 64 + lane] = acc[r];
    }
    // conv3's taps conv2's tail did not issue (it has K2 steps)
#pragma unroll
    for (int k = (K2 < 25 ? K2 : 25); k < K3; ++k) w3[k].load(wk3, wpl, k, tid);
    __syncthreads();   // (the ring and P1's reads are done)
    if (wk2g == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[((wid & 3) * 16 + r) * 64 + lane];
      // rows 8g + 4h + 0..3 of m block wm2 = pooled window 8 wm2 + 2g + h of
      // the 4 x 4 pool2 grid, channel 32 wn2 + l31
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int wn = 8 * wm2 + 2 * g + h;
        const int co = 32 * wn2 + l31;
        uint8_t rt;
        const float o = pool4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3], bias2, rt);
        lds_split3(P2 + ((wn >> 2) + 1) * P2_RS + ((wn & 3) + 1) * P2_CS + co, P2_PL, o);
        stg2[wn * 64 + co] = rt;
      }
    }
  }
  __syncthreads();   // P2 complete, the sums read
  w3[0].store(ring3, tid);
  w3[1].store(ring3 + W3_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(5);

  // ---- conv3: 9 taps on 16x16x32 ----
  {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, cor = {0.f, 0.f, 0.f, 0.f};
    const int r = lane & 15, kq = lane >> 4;
    const int win = r >> 2, y = 2 * (win >> 1) + ((r >> 1) & 1), x = 2 * (win & 1) + (r & 1);
    const int abase = y * P2_RS + x * P2_CS + 32 * wk3g + 8 * kq;
    const int bbase = (16 * wn3 + r) * W3_CW + 32 * wk3g + 8 * kq;
    bf16x8 av[2][3], bv[2][3];
    auto ops = [&](int t, int set) {
      const __bf16* wb = ring3 + (t % 3) * W3_SLOT;
      const __bf16* pa = P2 + (t / 3) * P2_RS + (t % 3) * P2_CS;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        av[set][p] = *reinterpret_cast<const bf16x8*>(pa + p * P2_PL + abase);
        bv[set][p] = *reinterpret_cast<const bf16x8*>(wb + p * W3_PL + bbase);
      }
    };
    ops(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + K3 < 9) w3[(t + K3) % K3].load(wk3, wpl, t + K3, tid);
      if (t + 1 < 9) ops(t + 1, (t + 1) & 1);
      const int c = t & 1;
      cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][2], bv[c][0], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][1], bv[c][1], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][0], bv[c][2], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][1], bv[c][0], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][0], bv[c][1], cor, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][0], bv[c][0], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < 9) w3[(t + 2) % K3].store(ring3 + ((t + 2) % 3) * W3_SLOT, tid);
      __syncthreads();
    }
    acc += cor;
    DDQ_STAMP(6);
    if (wk3g == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(wn3 * 4 + e) * 64 + lane] = acc[e];
    }
    __syncthreads();
    if (wk3g == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += red[(wn3 * 4 + e) * 64 + lane];
      // lane rows 4 kq + 0..3 = window kq of the 2 x 2 pool3 grid, channel
      // 16 wn3 + r: Caffe (B, 64, 2, 2) -- a wave writes 256 contiguous bytes
      const int co = 16 * wn3 + r;
      uint8_t rt;
      const float o = pool4(acc[0], acc[1], acc[2], acc[3], bias3, rt);
      a.pool3[z][((size_t)b * 64 + co) * 4 + kq] = o;
      if (q_tower && a.mask3) a.mask3[((size_t)b * 4 + kq) * 64 + co] = rt;
    }
  }
  // ---- the Q tower's pool1 / pool2 (split) and routing bytes (the backward's
  // inputs), 16-byte stores out of the images ----
  if (q_tower) {
    if (a.pool1s) {
      const int64_t E = (int64_t)a.B * 2048;
      for (int f = tid; f < 3 * 64 * 4; f += kThreads) {
        const int p = f / 256, r = f % 256, px = r >> 2, c = r & 3;
        const u32x4 v = *reinterpret_cast<const u32x4*>(P1 + p * P1_PL + ((px >> 3) + 2) * P1_RS +
                                                         ((px & 7) + 2) * P1_CS + 8 * c);
        *reinterpret_cast<u32x4*>(a.pool1s + p * E + ((size_t)b * 64 + px) * 32 + 8 * c) = v;
      }
    }
    if (a.pool2s) {
      const int64_t E = (int64_t)a.B * 1024;
      for (int f = tid; f < 3 * 16 * 8; f += kThreads) {
        const int p = f / 128, r = f % 128, px = r >> 3, c = r & 7;
        const u32x4 v = *reinterpret_cast<const u32x4*>(P2 + p * P2_PL + ((px >> 2) + 1) * P2_RS +
                                                         ((px & 3) + 1) * P2_CS + 8 * c);
        *reinterpret_cast<u32x4*>(a.pool2s + p * E + ((size_t)b * 16 + px) * 64 + 8 * c) = v;
      }
    }
    if (a.mask1 && tid < 128)
      reinterpret_cast<u32x4*>(a.mask1 + (size_t)b * 2048)[tid] = reinterpret_cast<const u32x4*>(stg1)[tid];
    if (a.mask2 && tid >= 128 && tid < 192)
      reinterpret_cast<u32x4*>(a.mask2 + (size_t)b * 1024)[tid - 128] =
          reinterpret_cast<const u32x4*>(stg2)[tid - 128];
  }
  DDQ_STAMP(7);
}


// ---------------------------------------------------------------------------
// K1, split form (B * nz <= 64): two workgroups per (image, tower), h = the
// half of conv2's and conv3's output channels each computes.  Both compute
// conv1 in full (conv2 needs all 32 of its channels); each streams half of
// conv2's and conv3's weights (307 KB instead of 571) and runs half their MFMA
// chains; the pool2 halves are exchanged through a two-workgroup meet
// (write-through stores, sc1 loads).  conv2 and conv3 on 16x16x32: conv2
// waves (m block of 16 pixels, n block of 16 channels) = 4 x 2, one 32-channel
// k step a tap; conv3 waves (n block, k step, tap parity) = 2 x 2 x 2 over a
// ring of tap pairs.
// ---------------------------------------------------------------------------
constexpr int Q1_CS = 48, Q1_RS = 576, Q1_PL = 12 * Q1_RS;             // pool1 image (MF 1)
constexpr int WH2_CW = 48, WH2_PL = 32 * WH2_CW, WH2_SLOT = 3 * WH2_PL; // conv2 half taps
constexpr int WH3_TAP = 3 * 32 * W3_CW;                                 // conv3 half tap
constexpr int WH3_SLOT = 2 * WH3_TAP;                                   // a pair of taps
constexpr int SOFF_RING3 = OFF_R;                                       // 3 x 30720
constexpr int SOFF_RED = SOFF_RING3;                  // 6 waves x 4 x 64 fp32, over the dead ring
constexpr int kFwdSmemS = SOFF_RING3 + 3 * WH3_SLOT * 2;               // (+ 2 KB static: book_block)
static_assert(3 * Q1_PL * 2 == 41472, "pool1 image");
constexpr int WH2P_SLOT = 2 * WH2_SLOT;                                // a pair of taps
static_assert(OFF_R + 3 * WH2P_SLOT * 2 <= kFwdSmemS && kFwdSmemS <= 160 * 1024, "split LDS");

// conv2 half taps: 3 planes x 32 co x 32 ci = 384 vectors (threads < 384)
struct WH2Tap {
  u32x4 r;
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int tap,
                                       int half, int tid) {
    const int f = tid < 384 ? tid : 383;
    const int p = f >> 7, q = f & 127, n = q >> 2, c8 = q & 3;
    r = *reinterpret_cast<const u32x4*>(wk + p * plane + ((32 * half + n) * 25 + tap) * 32 + 8 * c8);
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
    if (tid >= 384) return;
    const int p = tid >> 7, q = tid & 127, n = q >> 2, c8 = q & 3;
    *reinterpret_cast<u32x4*>(slot + p * WH2_PL + n * WH2_CW + 8 * c8) = r;
  }
};
// conv2 half tap pairs (taps 2s, 2s + 1; tap 25 does not exist: repeats 24)
struct WH2Pair {
  u32x4 r[2];
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int s,
                                       int half, int tid) {
    const int f = tid < 384 ? tid : 383;
    const int p = f >> 7, q = f & 127, n = q >> 2, c8 = q & 3;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tap = min(2 * s + u, 24);
      r[u] = *reinterpret_cast<const u32x4*>(wk + p * plane + ((32 * half + n) * 25 + tap) * 32 + 8 * c8);
    }
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
    if (tid >= 384) return;
    const int p = tid >> 7, q = tid & 127, n = q >> 2, c8 = q & 3;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<u32x4*>(slot + u * WH2_SLOT + p * WH2_PL + n * WH2_CW + 8 * c8) = r[u];
  }
};
// conv3 half tap pairs (taps 2s, 2s + 1): 2 x 3 x 32 x 64 ch = 1536 vectors,
// 3 a thread (tap 9 does not exist: its vectors repeat tap 8, unused)
struct WH3Pair {
  u32x4 r[3];
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int s,
                                       int half, int tid) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int f = tid + 512 * u;
      const int tp = f / 768, rem = f % 768, p = rem >> 8, n = (rem & 255) >> 3, c8 = rem & 7;
      const int tap = min(2 * s + tp, 8);
      r[u] = *reinterpret_cast<const u32x4*>(wk + p * plane + ((32 * half + n) * 9 + tap) * 64 + 8 * c8);
    }
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int f = tid + 512 * u;
      const int tp = f / 768, rem = f % 768, p = rem >> 8, n = (rem & 255) >> 3, c8 = rem & 7;
      *reinterpret_cast<u32x4*>(slot + tp * WH3_TAP + p * (32 * W3_CW) + n * W3_CW + 8 * c8) = r[u];
    }
  }
};

template <int K2, int K3>
__global__ __launch_bounds__(kThreads) void tower_fwd16s_kernel(const TowerArgs a) {
  static_assert(K2 >= 3 && K3 >= 3, "ring: step t + 2 is stored from registers at step t");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int bid = blockIdx.x;
  if (bid >= 2 * a.B * a.nz) {
    if (bid - 2 * a.B * a.nz < a.ntr) tower_transpose(a, bid - 2 * a.B * a.nz, smem);
    else book_block(a.bk);
    return;
  }
  DDQ_STAMP(0);
  const int half = bid & 1, pair = bid >> 1;         // the two halves: adjacent workgroups
  const int z = pair % a.nz, b = pair / a.nz;
  const bool q_tower = z == 0;
  const __bf16* __restrict__ wk1 = a.wks[z];
  const __bf16* __restrict__ wk2 = a.wks[z] + a.wks_off2;
  const __bf16* __restrict__ wk3 = a.wks[z] + a.wks_off3;
  const int64_t wpl = a.wks_plane;
  __bf16* P1 = reinterpret_cast<__bf16*>(smem + OFF_P1);
  __bf16* P2 = reinterpret_cast<__bf16*>(smem + OFF_P2);
  __bf16* patch = reinterpret_cast<__bf16*>(smem + OFF_PATCH);
  __bf16* w1s = reinterpret_cast<__bf16*>(smem + OFF_W1);
  __bf16* ring2 = reinterpret_cast<__bf16*>(smem + OFF_R);
  __bf16* ring3 = reinterpret_cast<__bf16*>(smem + SOFF_RING3);
  float* red = reinterpret_cast<float*>(smem + SOFF_RED);
  uint8_t* stg1 = reinterpret_cast<uint8_t*>(smem + OFF_STG1);
  uint8_t* stg2 = reinterpret_cast<uint8_t*>(smem + OFF_STG2);
  const int r16 = lane & 15, kq = lane >> 4;

  // ---- prologue (as tower_fwd16): frames + conv1 weights, then conv2's taps ----
  constexpr int NP = C1_PH * C1_PW;
  float4 fv[2];
  {
    const float* __restrict__ in = a.in[z];
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int f = tid + it * kThreads;
      const int py = f / C1_PW, px = f % C1_PW;
      const int gy = py - 3, gx = px - 3;
      fv[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (f < NP && px < kS + 6 && (unsigned)gy < (unsigned)kS && (unsigned)gx < (unsigned)kS)
        fv[it] = *reinterpret_cast<const float4*>(in + (((size_t)b * kS + gy) * kS + gx) * 4);
    }
  }
  constexpr int NW1 = 3 * kConv1WPlane / 8;
  constexpr int WIT = (NW1 + kThreads - 1) / kThreads;
  u32x4 wv[WIT];
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int f0 = tid + it * kThreads;
    const int f = f0 < NW1 ? f0 : NW1 - 1;
    const int p = f / (kConv1WPlane / 8), r = f % (kConv1WPlane / 8);
    wv[it] = *reinterpret_cast<const u32x4*>(wk1 + p * wpl + 8 * (size_t)r);
  }
  const float bias1 = a.bias1[z][l31];
  const int mb2 = wid & 3, nb2 = wid >> 2;          // conv2: 16-pixel m block, 16-channel n block
  const float bias2 = a.bias2[z][32 * half + 16 * nb2 + r16];
  const int wn3 = wid & 1, kk3 = (wid >> 1) & 1, tg3 = wid >> 2;
  const float bias3 = a.bias3[z][32 * half + 16 * wn3 + r16];
  WH2Pair w2[K2];
#pragma unroll
  for (int k = 0; k < K2; ++k) w2[k].load(wk2, wpl, k, half, tid);
  for (int f = tid; f < (3 * Q1_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(P1)[f] = u32x4{0u, 0u, 0u, 0u};
  for (int f = tid; f < (3 * P2_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(P2)[f] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int f = tid + it * kThreads;
    if (f < NP) {
      const int py = f / C1_PW, px = f % C1_PW;
      __bf16 q[4] = {(__bf16)fv[it].x, (__bf16)fv[it].y, (__bf16)fv[it].z, (__bf16)fv[it].w};
      *reinterpret_cast<uint2*>(patch + py * C1_RS + px * 4) = *reinterpret_cast<uint2*>(q);
    }
  }
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int f0 = tid + it * kThreads;
    if (f0 < NW1) {
      const int p = f0 / (kConv1WPlane / 8), r = f0 % (kConv1WPlane / 8);
      const int n = r / 28, q8 = r % 28;
      *reinterpret_cast<u32x4*>(w1s + (p * 32 + n) * C1_CW + 8 * q8) = wv[it];
    }
  }
  __syncthreads();
  DDQ_STAMP(1);

  // ---- conv1 (both halves, in full) ----
  {
    f32x16 acc, cor;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[r] = 0.f; cor[r] = 0.f; }
    const int m = wid * 32 + l31;
    const int win = m >> 2, dy = (m >> 1) & 1, dx = m & 1;
    const int wy = win >> 3, wx = win & 7;
    const int abase = (2 * wy + dy) * C1_RS + (2 * wx + dx + 2 * h) * 4;
    const int bbase = l31 * C1_CW + h * 8;
#pragma unroll
    for (int ky = 0; ky < 7; ++ky) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        bf16x8 bv[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bv[p] = *reinterpret_cast<const bf16x8*>(w1s + p * 32 * C1_CW + bbase + ky * 32 + 16 * g);
        typedef __attribute__((address_space(3))) const u32x2 lds_u2;
        typedef __attribute__((address_space(3))) const char lds_c;
        lds_u2* la = (lds_u2*)(patch + abase + ky * C1_RS + 16 * g);
        uint32_t hi_off = 8;
        asm volatile("" : "+v"(hi_off));
        const u32x2 lo = *la;
        const u32x2 hi = *(lds_u2*)((lds_c*)la + hi_off);
        u32x4 av4 = {lo[0], lo[1], hi[0], hi[1]};
        const bf16x8 av = *reinterpret_cast<bf16x8*>(&av4);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[2], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[1], cor, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv[0], acc, 0, 0, 0);
      }
    }
    acc += cor;
    DDQ_STAMP(2);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int wn = 8 * wid + 2 * g + h;
      uint8_t rt;
      const float o = pool4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3], bias1, rt);
      lds_split3(P1 + ((wn >> 3) + 2) * Q1_RS + ((wn & 7) + 2) * Q1_CS + l31, Q1_PL, o);
      stg1[wn * 32 + l31] = rt;
    }
  }
  __syncthreads();
  w2[0].store(ring2, tid);
  w2[1].store(ring2 + WH2P_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(3);

  // ---- conv2, channels [32 half, +32): 25 taps on 16x16x32 ----
  WH3Pair w3[K3];
  {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, cor = {0.f, 0.f, 0.f, 0.f};
    const int m = 16 * mb2 + r16;                   // pixel (window-major: 4 windows a block)
    const int win = m >> 2, y = 2 * (win >> 2) + ((m >> 1) & 1), x = 2 * (win & 3) + (m & 1);
    const int abase = y * Q1_RS + x * Q1_CS + 8 * kq;
    const int bbase = (16 * nb2 + r16) * WH2_CW + 8 * kq;
    // 13 steps of a tap pair (2s, 2s + 1): one barrier a pair
    bf16x8 av[2][2][3], bv[2][2][3];
    auto ops = [&](int st, int set) {
      const __bf16* wb = ring2 + (st % 3) * WH2P_SLOT;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = min(2 * st + u, 24);
        const __bf16* pa = P1 + (t / 5) * Q1_RS + (t % 5) * Q1_CS;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          av[set][u][p] = *reinterpret_cast<const bf16x8*>(pa + p * Q1_PL + abase);
          bv[set][u][p] = *reinterpret_cast<const bf16x8*>(wb + u * WH2_SLOT + p * WH2_PL + bbase);
        }
      }
    };
    constexpr int NS = 13;
    ops(0, 0);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      if (st + K2 < NS) {
        w2[(st + K2) % K2].load(wk2, wpl, st + K2, half, tid);
      } else if (st + K2 - NS < K3) {   // conv3's first tap pairs under conv2's last ones
        w3[st + K2 - NS].load(wk3, wpl, st + K2 - NS, half, tid);
      }
      if (st + 1 < NS) ops(st + 1, (st + 1) & 1);
      const int c = st & 1;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (2 * st + u >= 25) continue;
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][u][2], bv[c][u][0], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][u][1], bv[c][u][1], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][u][0], bv[c][u][2], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][u][1], bv[c][u][0], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][u][0], bv[c][u][1], cor, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][u][0], bv[c][u][0], acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (st + 2 < NS) w2[(st + 2) % K2].store(ring2 + ((st + 2) % 3) * WH2P_SLOT, tid);
      __syncthreads();
    }
    acc += cor;
#pragma unroll
    for (int k = (K2 < 13 ? K2 : 13); k < K3; ++k) w3[k].load(wk3, wpl, k, half, tid);
    DDQ_STAMP(4);
    // rows 4 kq + i = window 4 mb2 + kq of the 4 x 4 pool2 grid, channel
    // 32 half + 16 nb2 + r16: its half of P2 and of the routing bytes
    const int wn = 4 * mb2 + kq, co = 32 * half + 16 * nb2 + r16;
    uint8_t rt;
    const float o = pool4(acc[0], acc[1], acc[2], acc[3], bias2, rt);
    lds_split3(P2 + ((wn >> 2) + 1) * P2_RS + ((wn & 3) + 1) * P2_CS + co, P2_PL, o);
    stg2[wn * 64 + co] = rt;
  }
  __syncthreads();
  // ---- exchange the halves: ours out (write-through), meet, theirs in ----
  {
    __bf16* mine = a.xchg + ((int64_t)pair * 2 + half) * 1536;
    const __bf16* theirs = a.xchg + ((int64_t)pair * 2 + (half ^ 1)) * 1536;
    const int p = tid >> 6, px = (tid >> 2) & 15, c8 = tid & 3;        // tid < 192
    const __amdgpu_buffer_rsrc_t rm = wt_rsrc(mine, 3072);
    if (tid < 192) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(P2 + p * P2_PL + ((px >> 2) + 1) * P2_RS +
                                                       ((px & 3) + 1) * P2_CS + 32 * half + 8 * c8);
      __builtin_amdgcn_raw_buffer_store_b128(v, rm, (p * 128 + px * 8 + c8 * 2) * 8, 0, 16);
    }
    w3[0].store(ring3, tid);                         // (P1 / conv2's ring are dead)
    w3[1].store(ring3 + WH3_SLOT, tid);
    meet(a.pairc + pair, 2, a.timeout);   // (a failure: K2 / K4 see the sticky word)
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__bf16*>(theirs), (short)0, 3072, 0x00020000);
    if (tid < 192) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rt, (p * 128 + px * 8 + c8 * 2) * 8, 0, 16));
      *reinterpret_cast<u32x4*>(P2 + p * P2_PL + ((px >> 2) + 1) * P2_RS + ((px & 3) + 1) * P2_CS +
                                32 * (half ^ 1) + 8 * c8) = v;
    }
  }
  __syncthreads();
  DDQ_STAMP(5);

  // ---- conv3, channels [32 half, +32): tap pairs s = 0..4, tap 2s + tg3 ----
  {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, cor = {0.f, 0.f, 0.f, 0.f};
    const int win = r16 >> 2, y = 2 * (win >> 1) + ((r16 >> 1) & 1), x = 2 * (win & 1) + (r16 & 1);
    const int abase = y * P2_RS + x * P2_CS + 32 * kk3 + 8 * kq;
    const int bbase = tg3 * WH3_TAP + (16 * wn3 + r16) * W3_CW + 32 * kk3 + 8 * kq;
    bf16x8 av[2][3], bv[2][3];
    auto ops = [&](int s, int set) {
      const int t = min(2 * s + tg3, 8);
      const __bf16* wb = ring3 + (s % 3) * WH3_SLOT;
      const __bf16* pa = P2 + (t / 3) * P2_RS + (t % 3) * P2_CS;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        av[set][p] = *reinterpret_cast<const bf16x8*>(pa + p * P2_PL + abase);
        bv[set][p] = *reinterpret_cast<const bf16x8*>(wb + p * (32 * W3_CW) + bbase);
      }
    };
    ops(0, 0);
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      if (s + K3 < 5) w3[(s + K3) % K3].load(wk3, wpl, s + K3, half, tid);
      if (s + 1 < 5) ops(s + 1, (s + 1) & 1);
      const int c = s & 1;
      if (2 * s + tg3 < 9) {                         // (wave-uniform: tap 9 does not exist)
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][2], bv[c][0], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][1], bv[c][1], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][0], bv[c][2], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][1], bv[c][0], cor, 0, 0, 0);
        cor = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][0], bv[c][1], cor, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[c][0], bv[c][0], acc, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (s + 2 < 5) w3[(s + 2) % K3].store(ring3 + ((s + 2) % 3) * WH3_SLOT, tid);
      __syncthreads();
    }
    acc += cor;
    DDQ_STAMP(6);
    // the (k step, tap parity) partials of each n block meet in LDS, summed
    // in order (kk3, tg3) = (0,0) + (1,0) + (0,1) + (1,1)
    const int part = kk3 + 2 * tg3;
    if (part > 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(((part - 1) * 2 + wn3) * 4 + e) * 64 + lane] = acc[e];
    }
    __syncthreads();
    if (part == 0) {
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += red[((g * 2 + wn3) * 4 + e) * 64 + lane];
      const int co = 32 * half + 16 * wn3 + r16;
      uint8_t rt;
      const float o = pool4(acc[0], acc[1], acc[2], acc[3], bias3, rt);
      a.pool3[z][((size_t)b * 64 + co) * 4 + kq] = o;
      if (q_tower && a.mask3) a.mask3[((size_t)b * 4 + kq) * 64 + co] = rt;
    }
  }
  // ---- the Q tower's outputs: pool1 / pool2 (split) and pool1's routing
  // bytes by half 0 (both hold them in full), pool2's by each half for its
  // channels ----
  if (q_tower) {
    if (a.pool1s && half == 0) {
      const int64_t E = (int64_t)a.B * 2048;
      for (int f = tid; f < 3 * 64 * 4; f += kThreads) {
        const int p = f / 256, r = f % 256, px = r >> 2, c = r & 3;
        const u32x4 v = *reinterpret_cast<const u32x4*>(P1 + p * Q1_PL + ((px >> 3) + 2) * Q1_RS +
                                                         ((px & 7) + 2) * Q1_CS + 8 * c);
        *reinterpret_cast<u32x4*>(a.pool1s + p * E + ((size_t)b * 64 + px) * 32 + 8 * c) = v;
      }
    }
    if (a.pool2s && half == 0) {
      const int64_t E = (int64_t)a.B * 1024;
      for (int f = tid; f < 3 * 16 * 8; f += kThreads) {
        const int p = f / 128, r = f % 128, px = r >> 3, c = r & 7;
        const u32x4 v = *reinterpret_cast<const u32x4*>(P2 + p * P2_PL + ((px >> 2) + 1) * P2_RS +
                                                         ((px & 3) + 1) * P2_CS + 8 * c);
        *reinterpret_cast<u32x4*>(a.pool2s + p * E + ((size_t)b * 16 + px) * 64 + 8 * c) = v;
      }
    }
    if (a.mask1 && half == 0 && tid < 128)
      reinterpret_cast<u32x4*>(a.mask1 + (size_t)b * 2048)[tid] = reinterpret_cast<const u32x4*>(stg1)[tid];
    if (a.mask2 && tid >= 128 && tid < 160) {        // window w, 16-byte vector 2 half + v
      const int w = (tid - 128) >> 1, v = 2 * half + ((tid - 128) & 1);
      reinterpret_cast<u32x4*>(a.mask2 + (size_t)b * 1024)[w * 4 + v] =
          reinterpret_cast<const u32x4*>(stg2)[w * 4 + v];
    }
  }
  DDQ_STAMP(7);
}

}  // namespace sm16
}  // namespace ddq
