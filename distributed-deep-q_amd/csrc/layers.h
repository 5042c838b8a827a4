// Implicit-GEMM problem definitions for the deepq layers
// (models/deepq/train_val.prototxt:38-215), consumed by gemm.h.
//
// Device activation layout is NHWC fp32 (channels innermost, so every
// operand loader issues 16-byte loads along a contiguous channel run).
// Conv weights are read from a kernel-layout copy Wk[co][ky][kx][ci] that the
// apply kernel refreshes in the same pass that updates the canonical Caffe
// (co,ci,ky,kx) parameters.  fc4 / Q_out read the Caffe layout directly.
//
// The forward epilogue fuses bias + ReLU + 2x2/2 max-pool and emits an argmax
// byte per pooled element: 0..3 = in-window position of the FIRST maximum
// (Caffe's `>` scan), 4 = window max <= 0 (ReLU kills the gradient).  The GEMM
// row index of a forward conv enumerates pre-pool pixels window-major
// (4 consecutive rows = one 2x2 window), so a lane's 4 consecutive accumulator
// registers hold exactly one window and pooling needs no cross-lane traffic.
#pragma once
#include "gemm.h"

namespace ddq {

// ---------------------------------------------------------------------------
// conv forward: C[pixel][co] = sum_{ky,kx,ci} in[b][y+ky-P][x+kx-P][ci] * W[co][ci][ky][kx]
// M = B*H*W (window-major), N = COUT, K = KS*KS*CIN ordered (ky,kx,ci).
// z = tower (0 = Q on state, 1 = P on next_state).
// ---------------------------------------------------------------------------
template <int CIN, int COUT, int KS, int PAD>
struct ConvFwd {
  static constexpr bool kAK4 = true, kBK4 = true;
  struct KCtx {};
  __device__ KCtx ktile(int, int) const { return {}; }
  static constexpr int KC = KS * KS * CIN;
  int M, N, K, ksplit_len;
  int H, W;
  FastDiv fWp, fHp;                 // pooled grid (W/2, H/2)
  const float* in[2];               // NHWC (B,H,W,CIN)
  const float* wk[2];               // [COUT][KS][KS][CIN]
  const float* bias[2];             // [COUT]
  float* out[2];                    // pooled NHWC (B,H/2,W/2,COUT), or NCHW if nchw
  uint8_t* mask[2];                 // pooled argmax bytes (nullable), same layout
  int nchw;                         // 1: pooled output in Caffe (B,C,H/2,W/2) order
  FastDiv fHWp;                     // (H/2)*(W/2)

  struct ACtx { int b, y, x; bool ok; };
  __device__ ACtx actx(int, int m) const {
    ACtx c;
    c.ok = m < M;
    uint32_t q = (uint32_t)(c.ok ? m : 0) >> 2, w = (uint32_t)m & 3u, t, px, b, py;
    fWp.divmod(q, t, px);
    fHp.divmod(t, b, py);
    c.b = (int)b;
    c.y = 2 * (int)py + (int)(w >> 1);
    c.x = 2 * (int)px + (int)(w & 1);
    return c;
  }
  __device__ float4 loadA(int z, const ACtx& c, const KCtx&, int, int k) const {
    if (!c.ok || k >= K) return f4zero();
    const int tap = k / CIN, ci = k % CIN;
    const int ky = tap / KS, kx = tap % KS;
    const int yy = c.y + ky - PAD, xx = c.x + kx - PAD;
    if ((unsigned)yy >= (unsigned)H || (unsigned)xx >= (unsigned)W) return f4zero();
    return *reinterpret_cast<const float4*>((z ? in[1] : in[0]) + (((size_t)c.b * H + yy) * W + xx) * CIN + ci);
  }
  struct BCtx { int n; };
  __device__ BCtx bctx(int, int n) const { return {n}; }
  __device__ float4 loadB(int z, const BCtx&, const KCtx&, int k, int n) const {
    if (n >= N || k >= K) return f4zero();
    return *reinterpret_cast<const float4*>((z ? wk[1] : wk[0]) + (size_t)n * KC + k);
  }
  __device__ void epilogue(int z, int, int mb, int nb, const f32x16& acc, int lane) const {
    const int co = nb + (lane & 31);
    if (co >= N) return;
    const float bv = (z ? bias[1] : bias[0])[co];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int m = mb + 8 * g + 4 * (lane >> 5);
      if (m >= M) continue;
      const size_t q = (size_t)(m >> 2);
      // Caffe: top = conv + bias; ReLU in place; MAX pool first-max scan
      float v0 = acc[4 * g + 0] + bv, v1 = acc[4 * g + 1] + bv;
      float v2 = acc[4 * g + 2] + bv, v3 = acc[4 * g + 3] + bv;
      float mx = v0; int arg = 0;
      if (v1 > mx) { mx = v1; arg = 1; }
      if (v2 > mx) { mx = v2; arg = 2; }
      if (v3 > mx) { mx = v3; arg = 3; }
      const bool pos = mx > 0.f;
      size_t o = q * COUT + co;
      if (nchw) {
        uint32_t bb, pp;
        fHWp.divmod((uint32_t)q, bb, pp);
        o = ((size_t)bb * COUT + co) * fHWp.d + pp;
      }
      (z ? out[1] : out[0])[o] = pos ? mx : 0.f;
      uint8_t* mz = z ? mask[1] : mask[0];
      if (mz) mz[o] = (uint8_t)(pos ? arg : 4);
    }
  }
};

// ---------------------------------------------------------------------------
// conv weight gradient (+ bias gradient as an extra all-ones column):
// C[co][n] = sum_{pixel} dconv[pixel][co] * im2col(in)[pixel][n],  n < KC
// C[co][KC] = sum_{pixel} dconv[pixel][co]                     (bias diff)
// M = COUT, N = KC + 1, K = B*H*W pixels (plain (b,y,x) order), split-K over
// pixels into fp32 slabs part[split][COUT][NP] (reduced deterministically).
// ---------------------------------------------------------------------------
template <int CIN, int COUT, int KS, int PAD>
struct ConvWgrad {
  static constexpr bool kAK4 = false, kBK4 = false;
  static constexpr int KC = KS * KS * CIN;
  int M, N, K, ksplit_len;
  int H, W;
  FastDiv fW, fH;
  int rowtile;                      // 1: W % BK == 0 (host-checked): every K-tile lies in one image row
  // K-tile-uniform pixel decode (row tiles): the tile's image b, row y, first x
  struct KCtx { int b, y, x0, kb; };
  __device__ KCtx ktile(int, int kb) const {
    KCtx c{0, 0, 0, kb};
    if (rowtile) {
      uint32_t r, x0, b, y;
      fW.divmod((uint32_t)kb, r, x0);
      fH.divmod(r, b, y);
      c.b = (int)b; c.y = (int)y; c.x0 = (int)x0;
    }
    return c;
  }
  int NP;                           // slab row pitch
  const float* dconv;               // NHWC (B,H,W,COUT)
  const float* in;                  // NHWC (B,H,W,CIN)
  float* part;                      // [split][COUT][NP]

  struct ACtx { int m; };
  __device__ ACtx actx(int, int m) const { return {m}; }
  __device__ float4 loadA(int, const ACtx&, const KCtx&, int m, int k) const {
    if (k >= K || m >= M) return f4zero();
    return *reinterpret_cast<const float4*>(dconv + (size_t)k * COUT + m);
  }
  struct BCtx { int ky, kx, ci, kind; };
  __device__ BCtx bctx(int, int n) const {
    BCtx c;
    if (n < KC) {
      const int tap = n / CIN;
      c.ci = n % CIN; c.ky = tap / KS; c.kx = tap % KS; c.kind = 0;
    } else {
      c.ci = c.ky = c.kx = 0;
      c.kind = (n == KC) ? 1 : 2;
    }
    return c;
  }
  __device__ float4 loadB(int, const BCtx& c, const KCtx& kc, int k, int) const {
    if (k >= K || c.kind == 2) return f4zero();
    if (c.kind == 1) return f4(1.f, 0.f, 0.f, 0.f);
    uint32_t x, b, y;
    if (rowtile) {
      b = (uint32_t)kc.b; y = (uint32_t)kc.y;
      x = (uint32_t)(kc.x0 + (k - kc.kb));
    } else {
      uint32_t t;
      fW.divmod((uint32_t)k, t, x);
      fH.divmod(t, b, y);
    }
    const int yy = (int)y + c.ky - PAD, xx = (int)x + c.kx - PAD;
    if ((unsigned)yy >= (unsigned)H || (unsigned)xx >= (unsigned)W) return f4zero();
    return *reinterpret_cast<const float4*>(in + (((size_t)b * H + yy) * W + xx) * CIN + c.ci);
  }
  __device__ void epilogue(int, int split, int mb, int nb, const f32x16& acc, int lane) const {
    const int n = nb + (lane & 31);
    float* dst = part + (size_t)split * COUT * NP + n;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb + acc_row(r, lane);
      if (m < M) dst[(size_t)m * NP] = acc[r];
    }
  }
};

// ---------------------------------------------------------------------------
// conv data gradient w.r.t. this layer's input, fused with the previous
// layer's un-pool + ReLU mask:
// d_in[pixel][ci] = sum_{ky,kx,co} dconv[b][y+P-ky][x+P-kx][co] * W[co][ci][ky][kx]
// then prev_dconv[b][2y+dy][2x+dx][ci] = (prev_mask[pixel][ci] == 2dy+dx) ? d_in : 0
// M = B*H*W (plain order), N = CIN, K = KS*KS*COUT ordered (ky,kx,co).
// ---------------------------------------------------------------------------
template <int CIN, int COUT, int KS, int PAD>
struct ConvDgrad {
  static constexpr bool kAK4 = true, kBK4 = false;
  struct KCtx {};
  __device__ KCtx ktile(int, int) const { return {}; }
  int M, N, K, ksplit_len;
  int H, W;
  FastDiv fW, fH;
  const float* dconv;               // NHWC (B,H,W,COUT)
  const float* wk;                  // [COUT][KS][KS][CIN]
  const uint8_t* pmask;             // NHWC (B,H,W,CIN) argmax of previous pool
  float* pdconv;                    // NHWC (B,2H,2W,CIN)

  struct ACtx { int b, y, x; bool ok; };
  __device__ ACtx actx(int, int m) const {
    ACtx c;
    c.ok = m < M;
    uint32_t t, x, b, y;
    fW.divmod((uint32_t)(c.ok ? m : 0), t, x);
    fH.divmod(t, b, y);
    c.b = (int)b; c.y = (int)y; c.x = (int)x;
    return c;
  }
  __device__ float4 loadA(int, const ACtx& c, const KCtx&, int, int k) const {
    if (!c.ok || k >= K) return f4zero();
    const int tap = k / COUT, co = k % COUT;
    const int ky = tap / KS, kx = tap % KS;
    const int yy = c.y + PAD - ky, xx = c.x + PAD - kx;
    if ((unsigned)yy >= (unsigned)H || (unsigned)xx >= (unsigned)W) return f4zero();
    return *reinterpret_cast<const float4*>(dconv + (((size_t)c.b * H + yy) * W + xx) * COUT + co);
  }
  struct BCtx { int n; };
  __device__ BCtx bctx(int, int n) const { return {n}; }
  __device__ float4 loadB(int, const BCtx&, const KCtx&, int k, int n) const {
    if (k >= K || n >= N) return f4zero();
    const int tap = k / COUT, co = k % COUT;
    return *reinterpret_cast<const float4*>(wk + ((size_t)co * KS * KS + tap) * CIN + n);
  }
  __device__ void epilogue(int, int, int mb, int nb, const f32x16& acc, int lane) const {
    const int ci = nb + (lane & 31);
    if (ci >= N) return;
    const int W2 = 2 * W;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb + acc_row(r, lane);
      if (m >= M) continue;
      uint32_t t, x, b, y;
      fW.divmod((uint32_t)m, t, x);
      fH.divmod(t, b, y);
      const int mk = pmask[(size_t)m * CIN + ci];
      const float v = acc[r];
      float* base = pdconv + (((size_t)b * 2 * H + 2 * y) * W2 + 2 * x) * CIN + ci;
      base[0] = (mk == 0) ? v : 0.f;
      base[CIN] = (mk == 1) ? v : 0.f;
      base[(size_t)W2 * CIN] = (mk == 2) ? v : 0.f;
      base[(size_t)W2 * CIN + CIN] = (mk == 3) ? v : 0.f;
    }
  }
};

// ---------------------------------------------------------------------------
// fc4 forward, split-K: part[split][z][b][n] = sum_k x4[b][k] * W4[n][k]
// x4 = pool3 stored by conv3's epilogue in Caffe NCHW order (k = c*S4^2 + p),
// so both operands are contiguous.  M = B, N = 512, K = 64*S4^2.
// ---------------------------------------------------------------------------
struct FcFwd {
  static constexpr bool kAK4 = true, kBK4 = true;
  struct KCtx {};
  __device__ KCtx ktile(int, int) const { return {}; }
  int M, N, K, ksplit_len;
  const float* x[2];                // pool3 in Caffe NCHW order = the fc4 input row
  const float* w[2];                // (512, K) Caffe
  float* part;                      // [split][2][M][N]
  int nz;

  struct ACtx { int b; bool ok; };
  __device__ ACtx actx(int, int m) const { return {m, m < M}; }
  __device__ float4 loadA(int z, const ACtx& c, const KCtx&, int, int k) const {
    if (!c.ok || k >= K) return f4zero();
    return *reinterpret_cast<const float4*>((z ? x[1] : x[0]) + (size_t)c.b * K + k);
  }
  struct BCtx { int n; };
  __device__ BCtx bctx(int, int n) const { return {n}; }
  __device__ float4 loadB(int z, const BCtx&, const KCtx&, int k, int n) const {
    if (n >= N || k >= K) return f4zero();
    return *reinterpret_cast<const float4*>((z ? w[1] : w[0]) + (size_t)n * K + k);
  }
  __device__ void epilogue(int z, int split, int mb, int nb, const f32x16& acc, int lane) const {
    const int n = nb + (lane & 31);
    if (n >= N) return;
    float* dst = part + ((size_t)(split * nz + z) * M) * N + n;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb + acc_row(r, lane);
      if (m < M) dst[(size_t)m * N] = acc[r];
    }
  }
};

// ---------------------------------------------------------------------------
// fc4 data gradient fused with pool3 un-pool:
// dx4[b][k] = sum_n dh4[b][n] * W4[n][k]  (k Caffe order c*S4^2+p)
// -> dconv3[b][2py+dy][2px+dx][c] via mask3.  M = B, N = K4, K = 512.
// ---------------------------------------------------------------------------
struct FcDgrad {
  static constexpr bool kAK4 = true, kBK4 = false;
  struct KCtx {};
  __device__ KCtx ktile(int, int) const { return {}; }
  int M, N, K, ksplit_len;
  int s4, s4sq;
  FastDiv fS4sq, fS4;
  const float* dh4;                 // (B,512)
  const float* w4;                  // (512, N)
  const uint8_t* mask3;             // NCHW (B,64,S4,S4); unused when pooled
  float* dconv3;                    // NHWC (B,2S4,2S4,64), or pooled NHWC (B,S4,S4,64)
  int pooled;                       // as Fc4DgradArgs::pooled

  struct ACtx { int b; bool ok; };
  __device__ ACtx actx(int, int m) const { return {m, m < M}; }
  __device__ float4 loadA(int, const ACtx& c, const KCtx&, int, int k) const {
    if (!c.ok || k >= K) return f4zero();
    return *reinterpret_cast<const float4*>(dh4 + (size_t)c.b * K + k);
  }
  struct BCtx { int n; };
  __device__ BCtx bctx(int, int n) const { return {n}; }
  __device__ float4 loadB(int, const BCtx&, const KCtx&, int k, int n) const {
    if (k >= K || n >= N) return f4zero();
    return *reinterpret_cast<const float4*>(w4 + (size_t)k * N + n);
  }
  __device__ void epilogue(int, int, int mb, int nb, const f32x16& acc, int lane) const {
    const int kc = nb + (lane & 31);
    if (kc >= N) return;
    uint32_t ch, p, py, px;
    fS4sq.divmod((uint32_t)kc, ch, p);
    fS4.divmod(p, py, px);
    const int H3 = 2 * s4;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int b = mb + acc_row(r, lane);
      if (b >= M) continue;
      if (pooled) {
        dconv3[((size_t)b * s4sq + p) * 64 + ch] = acc[r];
        continue;
      }
      const int mk = mask3[(size_t)b * N + kc];          // NCHW: kc = ch*S4^2 + p
      const float v = acc[r];
      float* base = dconv3 + (((size_t)b * H3 + 2 * py) * H3 + 2 * px) * 64 + ch;
      base[0] = (mk == 0) ? v : 0.f;
      base[64] = (mk == 1) ? v : 0.f;
      base[(size_t)H3 * 64] = (mk == 2) ? v : 0.f;
      base[(size_t)H3 * 64 + 64] = (mk == 3) ? v : 0.f;
    }
  }
};

// ---------------------------------------------------------------------------
// fc4 weight gradient: gW4[n][k] = sum_b dh4[b][n] * x4[b][k], written
// straight into the flat gradient buffer (Caffe layout).  M = 512, N = K4, K = B.
// ---------------------------------------------------------------------------
struct FcWgrad {
  static constexpr bool kAK4 = false, kBK4 = false;
  struct KCtx {};
  __device__ KCtx ktile(int, int) const { return {}; }
  int M, N, K, ksplit_len;
  const float* dh4;                 // (B,512)
  const float* x;                   // pool3 of the Q tower, Caffe NCHW (B, K4)
  float* gw4;                       // (512, N)

  struct ACtx { int m; };
  __device__ ACtx actx(int, int m) const { return {m}; }
  __device__ float4 loadA(int, const ACtx&, const KCtx&, int m, int k) const {
    if (k >= K || m >= M) return f4zero();
    return *reinterpret_cast<const float4*>(dh4 + (size_t)k * M + m);
  }
  struct BCtx { int n; };
  __device__ BCtx bctx(int, int n) const { return {n}; }
  __device__ float4 loadB(int, const BCtx&, const KCtx&, int k, int n) const {
    if (k >= K || n >= N) return f4zero();
    return *reinterpret_cast<const float4*>(x + (size_t)k * N + n);
  }
  __device__ void epilogue(int, int, int mb, int nb, const f32x16& acc, int lane) const {
    const int n = nb + (lane & 31);
    if (n >= N) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb + acc_row(r, lane);
      if (m < M) gw4[(size_t)m * N + n] = acc[r];
    }
  }
};

}  // namespace ddq
