// The deepq16 step (small.h), launches K2..K4.  Included by kernels.hip after
// the update rules (apply_rule / ApplyArgs / ApplyTail) and the head's
// transposed-weight blocks (wkst_tap) it reuses.
#pragma once
#include "small.h"

namespace ddq {
namespace sm16 {

// ---------------------------------------------------------------------------
// K2: fc4 forward + head + fc4 backward + the fc4 / Q_out weight gradients
// and their apply (train_val.prototxt:159-215, 385-483), one launch.
//
// Workgroup j owns fc4 outputs n in [16 j, 16 j + 16) of both towers:
//   phase A  h4[z][b][n] = ReLU(b4 + W4[n] . pool3[z][b]) on f32 MFMA
//            (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 sums), and
//            its share of Q_out / P_out: qpart[j][z][b][a] = sum_n h4 W5[a][n]
//   fan-in   every workgroup needs every sample's Q_out / P_out (the target is
//            a max over P's actions): one arrival counter, write-through
//            partials and sc1 loads (MI355X_MICROARCH.md, inter-workgroup
//            visibility, table row 1), a bounded spin
//   phase B  Q_out, P_out, Q(s,a), target, loss (workgroup 0 writes them);
//            dQ; dh4 of its 16 units; the fc4 data gradient's partial over
//            them, dpart[j][b][k] = sum_n dh4[b][n] W4[n][k] (K3 sums the 32
//            partials in order); dW4 rows, db4, dW5 columns (and workgroup
//            0: db5) -- all final here, so the fused apply updates them here.
// The launch is 32 fc4 workgroups (all resident: one per CU at most).  (The
// transposed split weights K3 reads are made from the step's Q weights by K1's
// extra workgroups: kernels.hip tower_transpose.)
// ---------------------------------------------------------------------------
constexpr int kFcN = 16;                 // fc4 outputs per workgroup
constexpr int kFcBlk = 512 / kFcN;       // 32 workgroups
constexpr int kFcK = 256;                // fc4's K at S = 16 (64 x 2 x 2)
constexpr int kBC = 32;                  // images per chunk
constexpr int kXP = kFcK + 4;            // padded LDS row (floats)
constexpr int kMaxB = 256;
// LDS (floats): WS [2][16][kXP], XS [2][32][kXP], RED [2][2][4][64],
// H / DH [kMaxB][16] (h4 of Q, then dh4), QP [2][kMaxB][4], DQ [kMaxB][4]
constexpr int CH_WS = 0;
constexpr int CH_XS = CH_WS + 2 * kFcN * kXP;
constexpr int CH_RED = CH_XS + 2 * kBC * kXP;
constexpr int CH_H = CH_RED + 3 * 2 * 4 * 64;   // (k parts - 1 + tower slot) x half
constexpr int kHS = 18;                           // H / DH row stride: conflict-free operand
                                                  // reads (rows 18 floats apart, 64 banks)
constexpr int CH_DH = CH_H + kMaxB * kHS;
constexpr int CH_QP = CH_DH + kMaxB * kHS;
constexpr int CH_DQ = CH_QP + 2 * kMaxB * 4;
constexpr int CH_TMP = CH_DQ + kMaxB * 4;          // squared errors [kMaxB]
constexpr int CH_W5 = CH_TMP + kMaxB;             // Q's Q_out columns of the units [4][16]
constexpr int CH_PS = CH_W5 + 64;                 // theta / state of the 84 unit-sum params
constexpr int CH_MB = CH_PS + 2 * 96;             // the minibatch's action (4), reward, nonterm
constexpr int kChainSmemF = CH_MB + 6 * kMaxB;
constexpr int kChainSmem = kChainSmemF * 4;
static_assert(kChainSmem <= 160 * 1024, "K2 LDS");

struct ChainArgs {
  int B;
  const float* x[2];               // pool3 of each tower, Caffe (B, 256)
  const float* th[2];              // theta Q / P (flat Caffe layout)
  int64_t w4_off, b4_off, w5_off, b5_off;
  const float *action, *reward, *nonterm;
  float gamma;
  float* qpart;                    // [32][2][B][4]
  float* dpart;                    // [32][B][256]
  int32_t* sync;                   // [0..1] the fan-in's 64-bit counter, [2] sticky spin timeout,
                                   // [48] K1's (the pool2 halves' exchange)
  float *q_out, *p_out, *q_sa, *p_sa, *target, *loss;
  float* grad;                     // flat Q gradient
  int apply;                       // fused apply (flags latched by K1's book block)
  // B > 32: G = ceil(B / 32) image chunks, one per workgroup of a unit block
  // (32 G workgroups); the batch sums become per-chunk partials K4 sums in
  // chunk order: upart [G][32][96] (unit sums, db5, loss), w4part [G][512][256]
  int G;
  float* upart;
  float* w4part;
  int store_grad;                  // (unused: W4's gradient is always stored -- K4 applies it)
  ApplyArgs aa;
  ApplyTail at;
};

typedef float f32x4v __attribute__((ext_vector_type(4)));

// 16-byte sc1 load (misses L1; the producer's write-through bytes)
__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
  return __builtin_bit_cast(float4, v);
}

// Sum of 64 lanes' values in a fixed butterfly order (deterministic)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// NZ towers a workgroup: 1 (B <= 32: 64 workgroups, below) or 2 (B > 32: G
// chunks of 32 images, 32 G workgroups -- all resident with the launch's
// 159 KB of LDS only if each carries both towers)
template <int NZ>
__global__ __launch_bounds__(512) void fc4_chain16_kernel(const ChainArgs c) {
  extern __shared__ __attribute__((aligned(16))) float csm[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int bid = blockIdx.x;
  DDQ_STAMP(16);
  // one tower a workgroup: the P tower's kFcBlk G workgroups first (they run
  // phase A, publish their Q_out partials and leave without waiting, so the
  // Q tower's, which do wait, always find them dispatched), then the Q
  // tower's.  Unit block jb, image chunk cc: images [lo, hi) (G == 1: all)
  const int G = c.G, nH = kFcBlk * G;
  const bool ptower = NZ == 1 && bid < nH;
  const int zt = ptower ? 1 : 0, qb = ptower ? bid : (NZ == 1 ? bid - nH : bid);
  const int jb = qb % kFcBlk, cc = qb / kFcBlk;
  const int B = c.B, n0 = jb * kFcN;
  const int lo = G > 1 ? cc * kBC : 0, hi = G > 1 ? min(B, lo + kBC) : B;
  const int nch = (hi - lo + kBC - 1) / kBC;
  float* WS = csm + CH_WS;
  float* XS = csm + CH_XS;
  float* RED = csm + CH_RED;
  float* H = csm + CH_H;
  float* DH = csm + CH_DH;
  float* QP = csm + CH_QP;
  float* DQ = csm + CH_DQ;
  float* TMP = csm + CH_TMP;
  const int lr = lane & 15, kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rq = wt_rsrc(c.qpart, (uint32_t)(kFcBlk * 2 * B * 16));

  // ---- every global load of phase A's first chunk issued before the first
  // LDS store: the tower's W4 rows [n0, n0 + 16) (16 x 64 float4), the
  // chunk's pool3 rows (32 x 64 float4), the units' own fc4 bias and Q_out
  // columns ----
  float4 wv[2 * NZ], xv[4 * NZ];
  // (slot z of WS / XS: the tower, or 0 for a one-tower workgroup)
#pragma unroll
  for (int u = 0; u < 2 * NZ; ++u) {
    const int f = tid + u * 512;
    const int z = NZ == 2 ? f >> 10 : zt, n = (f >> 6) & 15, k4 = f & 63;
    wv[u] = *reinterpret_cast<const float4*>(c.th[z] + c.w4_off + (int64_t)(n0 + n) * kFcK + 4 * k4);
  }
  // phase A waves: NZ 2 (tower wz, image half wb, k half); NZ 1 (image half
  // wb, k quarter): wkq = the k part, of NKP
  constexpr int NKP = NZ == 2 ? 2 : 4, NKB = 8 / (NKP / 2);
  const int wz = NZ == 2 ? wid >> 2 : zt, wb = (wid >> 1) & 1;
  const int wkq = NZ == 2 ? (wid & 1) : 2 * (wid >> 2) + (wid & 1);
  const int wsl = NZ == 2 ? wz : 0;                  // the WS / XS slot of the wave's tower
#define DDQ_XLOAD(bb0)                                                                         \
  _Pragma("unroll") for (int u = 0; u < 4 * NZ; ++u) {                                         \
    const int f = tid + u * 512;                                                               \
    const int z = NZ == 2 ? f >> 11 : zt, b = (f >> 6) & 31, k4 = f & 63;                      \
    xv[u] = make_float4(0.f, 0.f, 0.f, 0.f);                                                   \
    if ((bb0) + b < hi) xv[u] = *reinterpret_cast<const float4*>(c.x[z] + (int64_t)((bb0) + b) * kFcK + 4 * k4); \
  }
#define DDQ_XSTORE()                                                                           \
  _Pragma("unroll") for (int u = 0; u < 4 * NZ; ++u) {                                         \
    const int f = tid + u * 512;                                                               \
    const int zs = NZ == 2 ? f >> 11 : 0, b = (f >> 6) & 31, k4 = f & 63;                      \
    *reinterpret_cast<float4*>(XS + (zs * kBC + b) * kXP + 4 * k4) = xv[u];                    \
  }
  DDQ_XLOAD(lo)
  float w5q = tid < 64 && !ptower ? c.th[0][c.w5_off + (tid >> 4) * 512 + n0 + (tid & 15)] : 0.f;
  // theta / optimizer state of the parameters the unit sums update (db4 and
  // dW5 columns of the units: q = 0..79; b5: q = 80..83, workgroup 0), read
  // now so phase B's updates wait on no load
  auto uparam = [&](int q) -> int64_t {
    return q < 80 ? ((q >> 4) == 0 ? c.b4_off + n0 + (q & 15) : c.w5_off + ((q >> 4) - 1) * 512 + n0 + (q & 15))
                  : c.b5_off + (q - 80);
  };
  float pth = 0.f, pst = 0.f;
  const bool ap0 = c.apply != 0 && G == 1 && !ptower;   // (G > 1: K4 applies the batch sums)
  // K1 failed its meeting: no update from this step (the word is read now,
  // used after the fan-in)
  const bool pois = ap0 && step_poisoned(c.sync + 48, nullptr);
  // the update's flags (latched by K1's book block), loaded now
  const bool first = ap0 && c.at.opt_init[2] != 0, sync = ap0 && c.at.opt_init[3] != 0;
  if (ap0 && tid < 84) {
    const int64_t i = uparam(tid);
    pth = c.at.theta[i];
    if (c.aa.rule != 0) pst = c.at.opt[i];
  }
  float b4v[4], w5v[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + 4 * kq + i;
    b4v[i] = c.th[wz][c.b4_off + n];
#pragma unroll
    for (int a = 0; a < 4; ++a) w5v[a][i] = c.th[wz][c.w5_off + a * 512 + n];
  }
#pragma unroll
  for (int u = 0; u < 2 * NZ; ++u) {
    const int f = tid + u * 512;
    const int zs = NZ == 2 ? f >> 10 : 0, n = (f >> 6) & 15, k4 = f & 63;
    *reinterpret_cast<float4*>(WS + (zs * kFcN + n) * kXP + 4 * k4) = wv[u];
  }
  if (!ptower) {
    if (tid < 64) csm[CH_W5 + tid] = w5q;
    if (tid < 84) { csm[CH_PS + tid] = pth; csm[CH_PS + 96 + tid] = pst; }
    for (int e = tid; e < 6 * B; e += 512)           // action one-hot, reward, non_terminal
      csm[CH_MB + e] = e < 4 * B ? c.action[e] : (e < 5 * B ? c.reward[e - 4 * B] : c.nonterm[e - 5 * B]);
  }

  // ---- phase A, chunk by chunk of 32 images ----
  for (int ch = 0; ch < nch; ++ch) {
    const int bb0 = lo + ch * kBC;
    if (ch) {
      __syncthreads();                             // previous chunk's XS reads done
      DDQ_XLOAD(bb0)
    }
    DDQ_XSTORE()
    __syncthreads();
    DDQ_STAMP(17);
    // wave: h[n][b] for its tower, 16 images, k part wkq of NKP; k-block k0:
    // MFMA step s pairs k = k0 + 4 kq + s of both operands
    f32x4v acc = {0.f, 0.f, 0.f, 0.f};
    const float* wrow = WS + (wsl * kFcN + lr) * kXP + 4 * kq;
    const float* xrow = XS + (wsl * kBC + 16 * wb + lr) * kXP + 4 * kq;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      const int k0 = (kFcK / NKP) * wkq + 16 * kb;
      const float4 av = *reinterpret_cast<const float4*>(wrow + k0);
      const float4 bv = *reinterpret_cast<const float4*>(xrow + k0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bv.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bv.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bv.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bv.w, acc, 0, 0, 0);
    }
    // RED slot of (k part p >= 1, this wave's tower slot and image half):
    // NZ 2 has p = 1 only, NZ 1 slot 0 only -- (p - 1 + slot) is unique
    auto rslot = [&](int p, int i) { return (((p - 1 + wsl) * 2 + wb) * 4 + i) * 64 + lane; };
    if (wkq != 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) RED[rslot(wkq, i)] = acc[i];
    }
    __syncthreads();
    if (wkq == 0) {
      // lane: units n = 4 kq + i, image b = 16 wb + lr (D rows / column)
      const int b = bb0 + 16 * wb + lr;
      float hv[4], q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // the k parts summed in order
        float v = acc[i];
#pragma unroll
        for (int p = 1; p < NKP; ++p) v += RED[rslot(p, i)];
        v += b4v[i];
        hv[i] = v > 0.f ? v : 0.f;                 // ReLU; dropout = identity (TEST phase)
#pragma unroll
        for (int a = 0; a < 4; ++a) q[a] += hv[i] * w5v[a][i];
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        q[a] += __shfl_xor(q[a], 16);
        q[a] += __shfl_xor(q[a], 32);
      }
      if (b < hi) {
        if (kq == 0)                               // write-through: the fan-in's hand-off
          wt_store4(rq, (uint32_t)((((jb * 2 + wz) * B + b) * 4) * 4), make_float4(q[0], q[1], q[2], q[3]));
        if (wz == 0)
#pragma unroll
          for (int i = 0; i < 4; ++i) H[b * kHS + 4 * kq + i] = hv[i];
      }
    }
  }
  DDQ_STAMP(18);
  if (ptower) {   // arrive (the partials drained, write-through) and leave
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(c.sync), (uint64_t)1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  meet(reinterpret_cast<uint64_t*>(c.sync), 2 * nH / NZ, c.sync + 2);
  const int32_t mword = ap0 ? meet_word(c.sync + 2) : 0;   // (consumed at the updates)
  DDQ_STAMP(19);

  // ---- phase B: every sample's Q_out / P_out (partials summed in j order) ----
  const int nbi = hi - lo;
  for (int p = tid; p < 2 * nbi; p += 512) {
    const int z = p / nbi, b = lo + p - z * nbi;
    float4 v[kFcBlk];
#pragma unroll
    for (int j = 0; j < kFcBlk; ++j) v[j] = ld_sc1_f4(rq, (uint32_t)((((j * 2 + z) * B + b) * 4) * 4));
    float4 s = v[0];
#pragma unroll
    for (int j = 1; j < kFcBlk; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
    // (Q_out's biases: nothing in this launch writes them -- at B <= 32 K4
    // applies their update, as it applies every batch sum's at B > 32)
    const float* th = c.th[z];
    s.x += th[c.b5_off + 0]; s.y += th[c.b5_off + 1]; s.z += th[c.b5_off + 2]; s.w += th[c.b5_off + 3];
    *reinterpret_cast<float4*>(QP + (z * kMaxB + b) * 4) = s;
  }
  __syncthreads();
  DDQ_STAMP(20);
  // head (ELTWISE PROD, SLICE, SUM, MAX, target, EUCLIDEAN_LOSS): as head_body
  for (int b = lo + tid; b < hi; b += 512) {
    const float* qp = QP + b * 4;
    const float* pp = QP + (kMaxB + b) * 4;
    const float* ac = csm + CH_MB + b * 4;
    float qs = qp[0] * ac[0];
    qs += qp[1] * ac[1];
    qs += qp[2] * ac[2];
    qs += qp[3] * ac[3];
    float ps = fmaxf(fmaxf(pp[0], pp[1]), fmaxf(pp[2], pp[3]));
    ps = ps * csm[CH_MB + 5 * B + b];
    const float tg = c.gamma * ps + 1.0f * csm[CH_MB + 4 * B + b];
    const float diff = qs - tg;
    const float gsc = diff / (float)B;
#pragma unroll
    for (int a = 0; a < 4; ++a) DQ[b * 4 + a] = ac[a] * gsc;
    TMP[b] = diff * diff;
    if (jb == 0) {
      c.q_sa[b] = qs; c.p_sa[b] = ps; c.target[b] = tg;
      *reinterpret_cast<float4*>(c.q_out + b * 4) = *reinterpret_cast<const float4*>(qp);
      *reinterpret_cast<float4*>(c.p_out + b * 4) = *reinterpret_cast<const float4*>(pp);
    }
  }
  __syncthreads();
  DDQ_STAMP(44);
  const bool ap = ap0 && !pois && mword == 0;
  // dh4 of the workgroup's units: (dQ W5) masked by h4 > 0 (ReLU backward)
  for (int e = lo * kFcN + tid; e < hi * kFcN; e += 512) {
    const int b = e >> 4, n = e & 15, eh = b * kHS + n;
    const float* w5 = csm + CH_W5 + n;
    const float* dq = DQ + b * 4;
    const float v = dq[0] * w5[0] + dq[1] * w5[16] + dq[2] * w5[32] + dq[3] * w5[48];
    DH[eh] = H[eh] > 0.f ? v : 0.f;
  }
  __syncthreads();
  DDQ_STAMP(45);
  // loss, db5 (workgroup 0) and db4, dW5 of the units: sums over the batch,
  // four threads a quantity (thread r of the four: samples r, r + 4, ... in
  // order), combined by two quad shuffles (fixed order, deterministic)
  {
    const int hq = jb == 0 ? 5 : 0, nq = hq + 5 * kFcN;
    const int qq = tid >> 2, r4 = tid & 3;
    const bool head = qq < hq;
    const int q = head ? qq : qq - hq;
    float v = 0.f;
    if (qq < nq) {
      if (head) {
        for (int b = lo + r4; b < hi; b += 4) v += q < 4 ? DQ[b * 4 + q] : TMP[b];
      } else {
        const int r = q >> 4, n = q & 15;            // r 0: db4, 1..4: dW5[r - 1]
        if (r == 0) {
          for (int b = lo + r4; b < hi; b += 4) v += DH[b * kHS + n];
        } else {
          for (int b = lo + r4; b < hi; b += 4) v += DQ[b * 4 + r - 1] * H[b * kHS + n];
        }
      }
    }
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    DDQ_STAMP(46);
    if (r4 == 0 && qq < nq && G > 1) {   // the chunk's partial: K4 sums the chunks
      c.upart[(cc * kFcBlk + jb) * 96 + (head ? (q == 4 ? 84 : 80 + q) : q)] = v;
    } else if (r4 == 0 && qq < nq) {
      if (head && q == 4) {
        *c.loss = v / (float)B / 2.f;
      } else {
        const int pq = head ? 80 + q : q;            // the preloaded parameter's slot
        const int64_t i = uparam(pq);
        const bool is_bias = head || (q >> 4) == 0;
        c.grad[i] = v;
        // (b5 -- head -- is read by every workgroup above: K4 updates it)
        if (ap && !head) {
          float st = (c.aa.rule != 0 && !first) ? csm[CH_PS + 96 + pq] : 0.f;
          const float th = apply_rule(c.aa, first, is_bias, csm[CH_PS + pq], v, st);
          c.at.theta[i] = th;
          if (c.aa.rule != 0) c.at.opt[i] = st;
          if (sync) c.at.thetaP[i] = th;
        }
      }
    }
  }
  DDQ_STAMP(21);
  // ---- dW4 rows [n0, +16) x 256 = sum_b dh4[b][n] x_Q[b][k] (f32 MFMA, K = b
  // in order: the fmaf chain of fc4_wgrad_sum), and the dpool3 partial
  // dpart[j][b][k] = sum_n dh4[b][n] W4[n][k] -- chunk by chunk of images ----
  // wave wid: dW4 k blocks 2 wid, 2 wid + 1; dpart tiles (b block, k block)
  f32x4v gw[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int ch = 0; ch < nch; ++ch) {
    const int bb0 = lo + ch * kBC;
    if (nch > 1) {                                 // reload the chunk's x_Q (one chunk: resident)
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int f = tid + u * 512;
        const int b = f >> 6, k4 = f & 63;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bb0 + b < hi) v = *reinterpret_cast<const float4*>(c.x[0] + (int64_t)(bb0 + b) * kFcK + 4 * k4);
        *reinterpret_cast<float4*>(XS + b * kXP + 4 * k4) = v;
      }
    }
    __syncthreads();
    const int nb = min(kBC, hi - bb0);
    // dW4: A[n][k = b] = DH[b][n], B[k = b][col] = x_Q[b][col]; the chunk's
    // 8 b quads' operands read first (rows past B are zero in XS, DH read 0)
    {
      float av8[8], bv8[8][2];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int b = 4 * q + kq;
        av8[q] = b < nb ? DH[(bb0 + b) * kHS + lr] : 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) bv8[q][u] = XS[b * kXP + 16 * (2 * wid + u) + lr];
      }
      // (transposed tile, A = x_Q, B = dh4: D rows = k, columns = n -- a lane's
      // 4 values are consecutive k of one row n, stored as one 16-byte vector)
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          gw[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv8[q][u], av8[q], gw[u], 0, 0, 0);
    }
    // dpart: tiles (b block bb, k block kb), 2 x 16 per chunk, 4 per wave
    float dav[4][4], dbv[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tI = wid * 4 + u, bbk = tI >> 4, kb = tI & 15;
      const int b = bb0 + 16 * bbk + lr;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int n = 4 * s + kq;
        dav[u][s] = b < hi ? DH[b * kHS + n] : 0.f;
        dbv[u][s] = WS[n * kXP + 16 * kb + lr];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tI = wid * 4 + u, bbk = tI >> 4, kb = tI & 15;
      if (16 * bbk >= nb) continue;                 // (wave-uniform)
      f32x4v d = {0.f, 0.f, 0.f, 0.f};
      // the transposed tile (A = the W4 columns, B = dh4; the same products in
      // the same n order): D rows = k 16 kb + 4 kq + i, column = image
      // 16 bbk + lr, so a lane holds 4 consecutive k of one image -- one
      // 16-byte store instead of four 4-byte ones
#pragma unroll
      for (int s = 0; s < 4; ++s) d = __builtin_amdgcn_mfma_f32_16x16x4f32(dbv[u][s], dav[u][s], d, 0, 0, 0);
      const int bi = bb0 + 16 * bbk + lr;
      if (bi < hi)
        *reinterpret_cast<float4*>(c.dpart + ((int64_t)jb * B + bi) * kFcK + 16 * kb + 4 * kq) =
            make_float4(d[0], d[1], d[2], d[3]);
    }
  }
  DDQ_STAMP(22);
  // ---- W4 rows: the gradient (K4's W4 blocks apply it: the rmsprop update's
  // correctly rounded divides and square roots, 8 a thread here, cost this
  // launch 2.8 us at its end; K4 has CUs free for them) ----
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int n = lr, k = 16 * (2 * wid + u) + 4 * kq;   // (w4_off % 4 == 0: launch check)
    const float4 v = make_float4(gw[u][0], gw[u][1], gw[u][2], gw[u][3]);
    if (G > 1) *reinterpret_cast<float4*>(c.w4part + ((int64_t)cc * 512 + n0 + n) * kFcK + k) = v;
    else *reinterpret_cast<float4*>(c.grad + c.w4_off + (int64_t)(n0 + n) * kFcK + k) = v;
  }
  DDQ_STAMP(23);
}


// ---------------------------------------------------------------------------
// K3: the Q tower's data gradients, one workgroup per image (train_val.
// prototxt:39-158 backward; conv1 has no bottom diff):
//   dpool3 = sum_j dpart[j] (fixed order) -> through pool3's routing bytes ->
//   dconv3 (split, LDS image, zero halo) -> conv3's data gradient on its
//   transposed + flipped split weights (K1's conv3 loop: the same
//   "forward" form on Wt[ci][8 - tap][co]) -> dpool2 -> pool2's routing ->
//   dconv2 (LDS image) -> conv2's data gradient (Wt[ci][24 - tap][co], 32x32x16,
//   four k groups) -> dpool1 -> pool1's routing -> dconv1 (LDS image) ->
//   conv1's weight gradient over the image's 256 pixels (split.h
//   w1_tile_wgrad's MFMA form: 7 tap rows x 16 pixel rows x 3 MFMAs) -> one
//   fp32 slab per image (K4 sums the B slabs in order).
// Also written (at the end, from LDS): dconv3 and dconv2 expanded + split,
// NHWC, the inputs of K4's conv3 / conv2 weight gradients.
// ---------------------------------------------------------------------------
// dconv3 image: 6 x 6 pixels x 80 (as K1's P2); dconv2 image: 12 x 12 pixels
// x 72 bf16 (64 channels + 8: odd 16-byte units), rows == 64 (mod 128)
constexpr int D2_CS = 72, D2_RS = 960, D2_PL = 12 * D2_RS;
constexpr int WD_CW = 72, WD_PL = 32 * WD_CW, WD_SLOT = 3 * WD_PL;   // conv2 dgrad ring (bf16)
// conv1 weight gradient (W1Fuse<8, 8, 512>): dconv1 image [3][16][16][32],
// frames halo [22][152] (pixel stride 4), units = tap rows
constexpr int X1_PL = 16 * 16 * 32, X1_IROW = 4 * 22 + 64;
// LDS map (bytes)
constexpr int B_D3 = 0;                                   // 20736
constexpr int B_M3 = 20736;                               // routing bytes: pool3 256
constexpr int B_M2 = B_M3 + 256;                          // pool2 1024
constexpr int B_M1 = B_M2 + 1024;                         // pool1 2048
constexpr int B_DP3 = B_M1 + 2048;                        // dpool3 (fp32 256) 1024
constexpr int B_SCR = B_DP3 + 1024;                       // 8 KB scratch (sums, k-group)
constexpr int B_RING3 = B_SCR + 8192;                     // 3 x 30720 (conv3 dgrad ring)
constexpr int B_D2 = B_RING3;                             // 69120 (after the conv3 dgrad)
constexpr int B_RING2 = B_D2 + 3 * D2_PL * 2;             // 3 x 13824
constexpr int B_RED2 = B_RING2;                           // 6 waves x 16 x 64 fp32 (after)
constexpr int B_X1 = B_RING2;                             // 49152 (after the conv2 dgrad)
constexpr int B_HALO = B_X1 + 3 * X1_PL * 2;              // 22 x 152 bf16 = 6688
constexpr int B_BIAS = B_HALO + 22 * X1_IROW * 2;         // 512 fp32
constexpr int kBwdSmem = B_BIAS + 512 * 4;
static_assert(B_RING3 + 3 * W3_SLOT * 2 <= kBwdSmem, "ring3");
static_assert(B_RING2 + 3 * WD_SLOT * 2 <= kBwdSmem && B_RED2 + 6 * 16 * 64 * 4 <= kBwdSmem, "ring2");
static_assert(kBwdSmem <= 160 * 1024, "K3 LDS");
static_assert(7 * 16 * 64 * 4 <= 3 * X1_PL * 2, "conv1 unit sums over the dconv1 image");

struct BwdArgs {
  int B;
  const float* dpart;              // [32][B][256] (K2)
  const uint8_t *mask1, *mask2, *mask3;
  const __bf16* wks;               // Q's split layouts: transposed data-gradient weights at
  int64_t wks_plane, wkst_off, wkst3_off;   // wkst_off (conv2), wkst3_off (conv3)
  const float* frames;             // state, fp32 NHWC (B, 16, 16, 4)
  __bf16* dconv3x;                 // split NHWC (B, 4, 4, 64), plane stride B * 1024
  __bf16* dconv2x;                 // split NHWC (B, 8, 8, 64), plane stride B * 4096
  float* w1part;                   // [B][32][w1_np] slabs, bias at column 196
  int w1_np;
};

// conv2 data-gradient weight taps: 3 planes x 32 ci x 64 co = 768 vectors
// (thread f, f + 512 for f < 256), rows of 8 vectors: 128-byte segments
struct WDTap {
  u32x4 r[2];
  static __device__ __forceinline__ void coords(int f, int& p, int& n, int& c8) {
    p = f >> 8;
    const int q = f & 255;
    n = q >> 3;
    c8 = q & 7;
  }
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int tap,
                                       int tid) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int f = s ? (tid < 256 ? tid + 512 : tid) : tid;
      int p, n, c8;
      coords(f, p, n, c8);
      r[s] = *reinterpret_cast<const u32x4*>(wk + p * plane + (n * 25 + tap) * 64 + 8 * c8);
    }
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s && tid >= 256) continue;
      const int f = tid + 512 * s;
      int p, n, c8;
      coords(f, p, n, c8);
      *reinterpret_cast<u32x4*>(slot + p * WD_PL + n * WD_CW + 8 * c8) = r[s];
    }
  }
};

template <int K3, int KD>
__global__ __launch_bounds__(kThreads) void tower_bwd16_kernel(const BwdArgs a) {
  static_assert(K3 >= 3 && KD >= 3, "ring: tap t + 2 is stored from registers at tap t");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int b = blockIdx.x, B = a.B;
  DDQ_STAMP(8);
  const __bf16* __restrict__ wt3 = a.wks + a.wkst3_off;
  const __bf16* __restrict__ wt2 = a.wks + a.wkst_off;
  const int64_t wpl = a.wks_plane;
  __bf16* D3 = reinterpret_cast<__bf16*>(smem + B_D3);
  __bf16* D2 = reinterpret_cast<__bf16*>(smem + B_D2);
  uint8_t* m3 = reinterpret_cast<uint8_t*>(smem + B_M3);
  uint8_t* m2 = reinterpret_cast<uint8_t*>(smem + B_M2);
  uint8_t* m1 = reinterpret_cast<uint8_t*>(smem + B_M1);
  float* dp3 = reinterpret_cast<float*>(smem + B_DP3);
  float* scr = reinterpret_cast<float*>(smem + B_SCR);
  __bf16* ring3 = reinterpret_cast<__bf16*>(smem + B_RING3);
  __bf16* ring2 = reinterpret_cast<__bf16*>(smem + B_RING2);
  float* red2 = reinterpret_cast<float*>(smem + B_RED2);
  __bf16* X = reinterpret_cast<__bf16*>(smem + B_X1);
  __bf16* halo = reinterpret_cast<__bf16*>(smem + B_HALO);
  float* bsm = reinterpret_cast<float*>(smem + B_BIAS);

  // ---- prologue: dpool3's partials (4 float4 a thread: group jg = tid / 64
  // sums j = 4 jg .. 4 jg + 3 of float4 k4 = tid % 64), the routing bytes,
  // then the first taps of both weight streams and the frames' halo ----
  float4 pv[4];
  {
    const int k4 = tid & 63, jg = tid >> 6;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      pv[u] = *reinterpret_cast<const float4*>(a.dpart + ((int64_t)(4 * jg + u) * B + b) * 256 + 4 * k4);
  }
  u32x4 mv = u32x4{0u, 0u, 0u, 0u};
  if (tid < 16) mv = reinterpret_cast<const u32x4*>(a.mask3 + (size_t)b * 256)[tid];
  else if (tid < 80) mv = reinterpret_cast<const u32x4*>(a.mask2 + (size_t)b * 1024)[tid - 16];
  else if (tid < 208) mv = reinterpret_cast<const u32x4*>(a.mask1 + (size_t)b * 2048)[tid - 80];
  W3Tap w3[K3];
#pragma unroll
  for (int k = 0; k < K3; ++k) w3[k].load(wt3, wpl, k, tid);
  // frames halo (conv1's weight gradient): 22 x 22 pixels, zero outside
  float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
  {
    const int hy = tid / 22, hx = tid - 22 * (tid / 22);
    const int gy = hy - 3, gx = hx - 3;
    if (tid < 484 && (unsigned)gy < 16u && (unsigned)gx < 16u)
      hv = *reinterpret_cast<const float4*>(a.frames + (((size_t)b * 16 + gy) * 16 + gx) * 4);
  }
  // zero the dconv3 image (halo + unrouted), then the sums
  for (int f = tid; f < (3 * P2_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(D3)[f] = u32x4{0u, 0u, 0u, 0u};
  {
    float4 s4 = pv[0];
#pragma unroll
    for (int u = 1; u < 4; ++u) { s4.x += pv[u].x; s4.y += pv[u].y; s4.z += pv[u].z; s4.w += pv[u].w; }
    reinterpret_cast<float4*>(scr)[tid] = s4;                 // [jg][k4]
  }
  if (tid < 16) reinterpret_cast<u32x4*>(m3)[tid] = mv;
  else if (tid < 80) reinterpret_cast<u32x4*>(m2)[tid - 16] = mv;
  else if (tid < 208) reinterpret_cast<u32x4*>(m1)[tid - 80] = mv;
  __syncthreads();
  if (tid < 256) {                                            // groups summed in order
    float v = scr[tid];
#pragma unroll
    for (int g = 1; g < 8; ++g) v += scr[g * 256 + tid];
    dp3[tid] = v;                                             // Caffe k = c * 4 + y * 2 + x
  }
  __syncthreads();
  // dconv3 (4 x 4 x 64): dpool3 at the routed quadrant of each 2 x 2 window
  for (int e = tid; e < 1024; e += kThreads) {
    const int px = e >> 6, c = e & 63, y = px >> 2, x = px & 3;
    const int pw = (y >> 1) * 2 + (x >> 1);
    const int q = ((y & 1) << 1) | (x & 1);
    const float v = m3[pw * 64 + c] == q ? dp3[c * 4 + pw] : 0.f;
    lds_split3(D3 + (y + 1) * P2_RS + (x + 1) * P2_CS + c, P2_PL, v);
  }
  w3[0].store(ring3, tid);
  w3[1].store(ring3 + W3_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(9);

  // ---- conv3 data gradient: 9 taps on 16x16x32 (K1's conv3 loop) ----
  WDTap wd[KD];
  const int wn3 = wid & 3, wk3g = wid >> 2;
  const int r16 = lane & 15, kq = lane >> 4;
  {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, cor = {0.f, 0.f, 0.f, 0.f};
    const int win = r16 >> 2, y = 2 * (win >> 1) + ((r16 >> 1) & 1), x = 2 * (win & 1) + (r16 & 1);
    const int abase = y * P2_RS + x * P2_CS + 32 * wk3g + 8 * kq;
    const int bbase = (16 * wn3 + r16) * W3_CW + 32 * wk3g + 8 * kq;
    bf16x8 av[2][3], bv[2][3];
    auto ops = [&](int t, int set) {
      const __bf16* wb = ring3 + (t % 3) * W3_SLOT;
      const __bf16* pa = D3 + (t / 3) * P2_RS + (t % 3) * P2_CS;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        av[set][p] = *reinterpret_cast<const bf16x8*>(pa + p * P2_PL + abase);
        bv[set][p] = *reinterpret_cast<const bf16x8*>(wb + p * W3_PL + bbase);
      }
    };
    ops(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + K3 < 9) {
        w3[(t + K3) % K3].load(wt3, wpl, t + K3, tid);
      } else if (t + K3 - 9 < KD) {   // conv2's data-gradient taps under conv3's last ones
        wd[t + K3 - 9].load(wt2, wpl, t + K3 - 9, tid);
      }
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
    DDQ_STAMP(10);
    if (wk3g == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) scr[(wn3 * 4 + e) * 64 + lane] = acc[e];
    }
    // zero the dconv2 image (over the dead ring) while the sums land
    for (int f = tid; f < (3 * D2_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(D2)[f] = u32x4{0u, 0u, 0u, 0u};
    // the conv2 data-gradient taps conv3's tail did not issue (it has K3 steps)
#pragma unroll
    for (int k = (K3 < 9 ? K3 : 9); k < KD; ++k) wd[k].load(wt2, wpl, k, tid);
    __syncthreads();
    if (wk3g == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += scr[(wn3 * 4 + e) * 64 + lane];
      // lane: dpool2 at pool2 pixels of window kq (rows 4 kq + i), channel
      // 16 wn3 + r16 -> the routed quadrant of its 2 x 2 conv2-output window
      const int c = 16 * wn3 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int y = 2 * (kq >> 1) + (i >> 1), x = 2 * (kq & 1) + (i & 1);
        const int q = m2[(y * 4 + x) * 64 + c];
        if (q < 4)
          lds_split3(D2 + (2 * y + (q >> 1) + 2) * D2_RS + (2 * x + (q & 1) + 2) * D2_CS + c, D2_PL,
                     acc[i]);
      }
    }
  }
  __syncthreads();
  wd[0].store(ring2, tid);
  wd[1].store(ring2 + WD_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(11);

  // ---- conv2 data gradient: 25 taps, 32x32x16; waves (m block, k step) =
  // 2 x 4: a tap's 64 co are four 16-channel k steps ----
  {
    const int wm = wid & 1, wkg = wid >> 1;
    f32x16 acc, cor;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[r] = 0.f; cor[r] = 0.f; }
    const int m = 32 * wm + l31;
    const int win = m >> 2, dy = (m >> 1) & 1, dx = m & 1;
    const int y = 2 * (win >> 2) + dy, x = 2 * (win & 3) + dx;
    const int abase = y * D2_RS + x * D2_CS + 16 * wkg + 8 * h;
    const int bbase = l31 * WD_CW + 16 * wkg + 8 * h;
    bf16x8 av[2][3], bv[2][3];
    auto ops = [&](int t, int set) {
      const __bf16* wb = ring2 + (t % 3) * WD_SLOT;
      const __bf16* pa = D2 + (t / 5) * D2_RS + (t % 5) * D2_CS;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        av[set][p] = *reinterpret_cast<const bf16x8*>(pa + p * D2_PL + abase);
        bv[set][p] = *reinterpret_cast<const bf16x8*>(wb + p * WD_PL + bbase);
      }
    };
    ops(0, 0);
#pragma unroll
    for (int t = 0; t < 25; ++t) {
      if (t + KD < 25) wd[(t + KD) % KD].load(wt2, wpl, t + KD, tid);
      if (t + 1 < 25) ops(t + 1, (t + 1) & 1);
      const int c = t & 1;
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][2], bv[c][0], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][1], bv[c][1], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][0], bv[c][2], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][1], bv[c][0], cor, 0, 0, 0);
      cor = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][0], bv[c][1], cor, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[c][0], bv[c][0], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < 25) wd[(t + 2) % KD].store(ring2 + ((t + 2) % 3) * WD_SLOT, tid);
      __syncthreads();
    }
    acc += cor;
    DDQ_STAMP(12);
    // four k groups meet in LDS, summed in order 0 + 1 + 2 + 3 by group 0
    if (wkg > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red2[(((wkg - 1) * 2 + wm) * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    // (the ring is dead: its region becomes the dconv1 image after the sums)
    float bsum = 0.f;
    if (wkg == 0) {
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += red2[((g * 2 + wm) * 16 + r) * 64 + lane];
    }
    __syncthreads();
    for (int f = tid; f < (3 * X1_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(X)[f] = u32x4{0u, 0u, 0u, 0u};
    {   // the frames' halo (fp32 -> bf16 exact), pixel stride 4 bf16
      if (tid < 484) {
        const int hy = tid / 22, hx = tid - 22 * (tid / 22);
        __bf16 q4[4] = {(__bf16)hv.x, (__bf16)hv.y, (__bf16)hv.z, (__bf16)hv.w};
        *reinterpret_cast<uint2*>(halo + hy * X1_IROW + 4 * hx) = *reinterpret_cast<uint2*>(q4);
      }
    }
    __syncthreads();
    if (wkg == 0) {
      // lane: dpool1 at rows 8g + 4h + i of m block wm (window-major pixels of
      // the 8 x 8 pool1 grid), channel l31 -> pool1's routed quadrant of dconv1
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int mm = 32 * wm + 8 * g + 4 * h + i;
          const int wn = mm >> 2;
          const int y = 2 * (wn >> 2) + ((mm >> 1) & 1), x = 2 * (wn & 3) + (mm & 1);
          const int q = m1[(y * 8 + x) * 32 + l31];
          if (q < 4) {
            const float v = acc[4 * g + i];
            bsum += v;
            lds_split3(X + ((2 * y + (q >> 1)) * 16 + 2 * x + (q & 1)) * 32 + l31, X1_PL, v);
          }
        }
    }
    bsm[tid] = bsum;
  }
  __syncthreads();
  DDQ_STAMP(13);

  // ---- conv1's weight gradient (split.h w1_tile_wgrad, one 16-pixel segment
  // per row): wave u < 7 = tap row ky, 16 conv1 rows x 3 MFMAs ----
  {
    const int gq = lane >> 4, iq = (lane & 15) >> 2, ip = lane & 3;
    const int pix0 = 8 * (gq >> 1) + iq;
    const int chn = 16 * (gq & 1) + 4 * ip;
    f32x16 wacc;
#pragma unroll
    for (int e = 0; e < 16; ++e) wacc[e] = 0.f;
    if (wid < 7) {
      const int ky = wid;
      const __bf16* pa0 = X + pix0 * 32 + chn;
      const __bf16* pb0 = halo + ky * X1_IROW + 4 * pix0 + chn;
#pragma unroll 4
      for (int row = 0; row < 16; ++row) {
        bf16x8 av[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const __bf16* pa = pa0 + p * X1_PL + row * 16 * 32;
          av[p] = tr_pair(pa, pa + 4 * 32);
        }
        const __bf16* pb = pb0 + row * X1_IROW;
        const bf16x8 bv = tr_pair(pb, pb + 16);
        wacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv, wacc, 0, 0, 0);
        wacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv, wacc, 0, 0, 0);
        wacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv, wacc, 0, 0, 0);
      }
    }
    __syncthreads();                                  // X / halo reads done
    float* ured = reinterpret_cast<float*>(X);        // [7][16][64]
    if (wid < 7) {
#pragma unroll
      for (int e = 0; e < 16; ++e) ured[(wid * 16 + e) * 64 + lane] = wacc[e];
    }
    __syncthreads();
    // the image's slab, 16-byte write-through stores: item = (ky, row r,
    // half h2, columns 4q..4q+3 < 28); rows co = (r & 3) + 8 (r >> 2) + 4 h2
    const uint32_t slab = (uint32_t)b * 32u * (uint32_t)a.w1_np;
    const __amdgpu_buffer_rsrc_t rs =
        wt_rsrc(a.w1part, (uint32_t)((size_t)B * 32u * (uint32_t)a.w1_np * 4));
    for (int f = tid; f < 7 * 16 * 14; f += kThreads) {
      const int ky = f / 224, rem = f - ky * 224;
      const int r = rem / 14, g = rem - r * 14, h2 = g / 7, q = g - h2 * 7;
      const float4 v = *reinterpret_cast<const float4*>(ured + (ky * 16 + r) * 64 + 32 * h2 + 4 * q);
      const int co = (r & 3) + 8 * (r >> 2) + 4 * h2;
      wt_store4(rs, (slab + (uint32_t)(co * a.w1_np + ky * 28 + 4 * q)) * 4, v);
    }
    if (tid < 32) {   // bias: the lanes of channel tid, k-group-0 waves in order
      float v = 0.f;
      for (int w = 0; w < 2; ++w) v += bsm[w * 64 + tid] + bsm[w * 64 + 32 + tid];
      wt_store(rs, (slab + (uint32_t)(tid * a.w1_np + 196)) * 4, v);
    }
  }
  // ---- dconv3 / dconv2 expanded + split, NHWC, out of the images ----
  {
    const int64_t E3 = (int64_t)B * 1024, E2 = (int64_t)B * 4096;
    for (int f = tid; f < 3 * 16 * 8; f += kThreads) {
      const int p = f / 128, r = f % 128, px = r >> 3, c = r & 7;
      const u32x4 v = *reinterpret_cast<const u32x4*>(D3 + p * P2_PL + ((px >> 2) + 1) * P2_RS +
                                                       ((px & 3) + 1) * P2_CS + 8 * c);
      *reinterpret_cast<u32x4*>(a.dconv3x + p * E3 + ((size_t)b * 16 + px) * 64 + 8 * c) = v;
    }
    for (int f = tid; f < 3 * 64 * 8; f += kThreads) {
      const int p = f / 512, r = f % 512, px = r >> 3, c = r & 7;
      const u32x4 v = *reinterpret_cast<const u32x4*>(D2 + p * D2_PL + ((px >> 3) + 2) * D2_RS +
                                                       ((px & 7) + 2) * D2_CS + 8 * c);
      *reinterpret_cast<u32x4*>(a.dconv2x + p * E2 + ((size_t)b * 64 + px) * 64 + 8 * c) = v;
    }
  }
  DDQ_STAMP(14);
}


// K3, split form (2 B <= 256 workgroups): two workgroups per image, h = the
// half of conv2's data-gradient channels (conv1's output channels) each
// computes -- and so of conv1's weight-gradient rows.  Both compute conv3's
// data gradient in full (no exchange: conv2's data gradient needs all of
// dconv2).  conv2's data gradient on 16x16x32: waves (m block of 16 pixels,
// 32-channel k step) = 4 x 2; the dconv2 image at pixel stride 80 (MF 1).
constexpr int DS_CS = 80;                                              // dconv2 image (MF 1)
constexpr int WDH_CW = 80, WDH_PL = 16 * WDH_CW, WDH_SLOT = 3 * WDH_PL;  // conv2 dgrad half taps
constexpr int WDHP_SLOT = 2 * WDH_SLOT;                                // a pair of taps
constexpr int BS_RED2 = B_RING2;                                      // (over the dead ring)
static_assert(12 * DS_CS <= D2_RS && B_RING2 + 3 * WDHP_SLOT * 2 <= B_HALO, "K3 split LDS");

// conv2 data-gradient half tap pairs (taps 2s, 2s + 1; 25 repeats 24)
struct WDHPair {
  u32x4 r[2];
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int s,
                                       int half, int tid) {
    const int f = tid < 384 ? tid : 383;
    const int p = f >> 7, q = f & 127, n = q >> 3, c8 = q & 7;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int tap = min(2 * s + u, 24);
      r[u] = *reinterpret_cast<const u32x4*>(wk + p * plane + ((16 * half + n) * 25 + tap) * 64 + 8 * c8);
    }
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
    if (tid >= 384) return;
    const int p = tid >> 7, q = tid & 127, n = q >> 3, c8 = q & 7;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<u32x4*>(slot + u * WDH_SLOT + p * WDH_PL + n * WDH_CW + 8 * c8) = r[u];
  }
};
// conv2 data-gradient half taps: 3 planes x 16 ci x 64 co = 384 vectors
struct WDHTap {
  u32x4 r;
  __device__ __forceinline__ void load(const __bf16* __restrict__ wk, int64_t plane, int tap,
                                       int half, int tid) {
    const int f = tid < 384 ? tid : 383;
    const int p = f >> 7, q = f & 127, n = q >> 3, c8 = q & 7;
    r = *reinterpret_cast<const u32x4*>(wk + p * plane + ((16 * half + n) * 25 + tap) * 64 + 8 * c8);
  }
  __device__ __forceinline__ void store(__bf16* slot, int tid) const {
    if (tid >= 384) return;
    const int p = tid >> 7, q = tid & 127, n = q >> 3, c8 = q & 7;
    *reinterpret_cast<u32x4*>(slot + p * WDH_PL + n * WDH_CW + 8 * c8) = r;
  }
};

template <int K3, int KD>
__global__ __launch_bounds__(kThreads) void tower_bwd16s_kernel(const BwdArgs a) {
  static_assert(K3 >= 3 && KD >= 3, "ring: tap t + 2 is stored from registers at tap t");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x >> 1, half = blockIdx.x & 1, B = a.B;
  DDQ_STAMP(8);
  const __bf16* __restrict__ wt3 = a.wks + a.wkst3_off;
  const __bf16* __restrict__ wt2 = a.wks + a.wkst_off;
  const int64_t wpl = a.wks_plane;
  __bf16* D3 = reinterpret_cast<__bf16*>(smem + B_D3);
  __bf16* D2 = reinterpret_cast<__bf16*>(smem + B_D2);
  uint8_t* m3 = reinterpret_cast<uint8_t*>(smem + B_M3);
  uint8_t* m2 = reinterpret_cast<uint8_t*>(smem + B_M2);
  uint8_t* m1 = reinterpret_cast<uint8_t*>(smem + B_M1);
  float* dp3 = reinterpret_cast<float*>(smem + B_DP3);
  float* scr = reinterpret_cast<float*>(smem + B_SCR);
  __bf16* ring3 = reinterpret_cast<__bf16*>(smem + B_RING3);
  __bf16* ring2 = reinterpret_cast<__bf16*>(smem + B_RING2);
  float* red2 = reinterpret_cast<float*>(smem + BS_RED2);
  __bf16* X = reinterpret_cast<__bf16*>(smem + B_X1);
  __bf16* halo = reinterpret_cast<__bf16*>(smem + B_HALO);
  float* bsm = reinterpret_cast<float*>(smem + B_BIAS);

  // ---- prologue: dpool3's partials (4 float4 a thread: group jg = tid / 64
  // sums j = 4 jg .. 4 jg + 3 of float4 k4 = tid % 64), the routing bytes,
  // then the first taps of both weight streams and the frames' halo ----
  float4 pv[4];
  {
    const int k4 = tid & 63, jg = tid >> 6;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      pv[u] = *reinterpret_cast<const float4*>(a.dpart + ((int64_t)(4 * jg + u) * B + b) * 256 + 4 * k4);
  }
  u32x4 mv = u32x4{0u, 0u, 0u, 0u};
  if (tid < 16) mv = reinterpret_cast<const u32x4*>(a.mask3 + (size_t)b * 256)[tid];
  else if (tid < 80) mv = reinterpret_cast<const u32x4*>(a.mask2 + (size_t)b * 1024)[tid - 16];
  else if (tid < 208) mv = reinterpret_cast<const u32x4*>(a.mask1 + (size_t)b * 2048)[tid - 80];
  W3Tap w3[K3];
#pragma unroll
  for (int k = 0; k < K3; ++k) w3[k].load(wt3, wpl, k, tid);
  // frames halo (conv1's weight gradient): 22 x 22 pixels, zero outside
  float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
  {
    const int hy = tid / 22, hx = tid - 22 * (tid / 22);
    const int gy = hy - 3, gx = hx - 3;
    if (tid < 484 && (unsigned)gy < 16u && (unsigned)gx < 16u)
      hv = *reinterpret_cast<const float4*>(a.frames + (((size_t)b * 16 + gy) * 16 + gx) * 4);
  }
  // zero the dconv3 image (halo + unrouted), then the sums
  for (int f = tid; f < (3 * P2_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(D3)[f] = u32x4{0u, 0u, 0u, 0u};
  {
    float4 s4 = pv[0];
#pragma unroll
    for (int u = 1; u < 4; ++u) { s4.x += pv[u].x; s4.y += pv[u].y; s4.z += pv[u].z; s4.w += pv[u].w; }
    reinterpret_cast<float4*>(scr)[tid] = s4;                 // [jg][k4]
  }
  if (tid < 16) reinterpret_cast<u32x4*>(m3)[tid] = mv;
  else if (tid < 80) reinterpret_cast<u32x4*>(m2)[tid - 16] = mv;
  else if (tid < 208) reinterpret_cast<u32x4*>(m1)[tid - 80] = mv;
  __syncthreads();
  if (tid < 256) {                                            // groups summed in order
    float v = scr[tid];
#pragma unroll
    for (int g = 1; g < 8; ++g) v += scr[g * 256 + tid];
    dp3[tid] = v;                                             // Caffe k = c * 4 + y * 2 + x
  }
  __syncthreads();
  // dconv3 (4 x 4 x 64): dpool3 at the routed quadrant of each 2 x 2 window
  for (int e = tid; e < 1024; e += kThreads) {
    const int px = e >> 6, c = e & 63, y = px >> 2, x = px & 3;
    const int pw = (y >> 1) * 2 + (x >> 1);
    const int q = ((y & 1) << 1) | (x & 1);
    const float v = m3[pw * 64 + c] == q ? dp3[c * 4 + pw] : 0.f;
    lds_split3(D3 + (y + 1) * P2_RS + (x + 1) * P2_CS + c, P2_PL, v);
  }
  w3[0].store(ring3, tid);
  w3[1].store(ring3 + W3_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(9);

  // ---- conv3 data gradient: 9 taps on 16x16x32 (K1's conv3 loop) ----
  WDHPair wd[KD];
  const int wn3 = wid & 3, wk3g = wid >> 2;
  const int r16 = lane & 15, kq = lane >> 4;
  {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, cor = {0.f, 0.f, 0.f, 0.f};
    const int win = r16 >> 2, y = 2 * (win >> 1) + ((r16 >> 1) & 1), x = 2 * (win & 1) + (r16 & 1);
    const int abase = y * P2_RS + x * P2_CS + 32 * wk3g + 8 * kq;
    const int bbase = (16 * wn3 + r16) * W3_CW + 32 * wk3g + 8 * kq;
    bf16x8 av[2][3], bv[2][3];
    auto ops = [&](int t, int set) {
      const __bf16* wb = ring3 + (t % 3) * W3_SLOT;
      const __bf16* pa = D3 + (t / 3) * P2_RS + (t % 3) * P2_CS;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        av[set][p] = *reinterpret_cast<const bf16x8*>(pa + p * P2_PL + abase);
        bv[set][p] = *reinterpret_cast<const bf16x8*>(wb + p * W3_PL + bbase);
      }
    };
    ops(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + K3 < 9) {
        w3[(t + K3) % K3].load(wt3, wpl, t + K3, tid);
      } else if (t + K3 - 9 < KD) {   // conv2's data-gradient taps under conv3's last ones
        wd[t + K3 - 9].load(wt2, wpl, t + K3 - 9, half, tid);
      }
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
    DDQ_STAMP(10);
    if (wk3g == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) scr[(wn3 * 4 + e) * 64 + lane] = acc[e];
    }
    // zero the dconv2 image (over the dead ring) while the sums land
    for (int f = tid; f < (3 * D2_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(D2)[f] = u32x4{0u, 0u, 0u, 0u};
    // the conv2 data-gradient taps conv3's tail did not issue (it has K3 steps)
#pragma unroll
    for (int k = (K3 < 9 ? K3 : 9); k < KD; ++k) wd[k].load(wt2, wpl, k, half, tid);   // (pairs)
    __syncthreads();
    if (wk3g == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += scr[(wn3 * 4 + e) * 64 + lane];
      // lane: dpool2 at pool2 pixels of window kq (rows 4 kq + i), channel
      // 16 wn3 + r16 -> the routed quadrant of its 2 x 2 conv2-output window
      const int c = 16 * wn3 + r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int y = 2 * (kq >> 1) + (i >> 1), x = 2 * (kq & 1) + (i & 1);
        const int q = m2[(y * 4 + x) * 64 + c];
        if (q < 4)
          lds_split3(D2 + (2 * y + (q >> 1) + 2) * D2_RS + (2 * x + (q & 1) + 2) * DS_CS + c, D2_PL,
                     acc[i]);
      }
    }
  }
  __syncthreads();
  wd[0].store(ring2, tid);
  wd[1].store(ring2 + WDHP_SLOT, tid);
  __syncthreads();
  DDQ_STAMP(11);

  // ---- conv2 data gradient, channels [16 half, +16): 25 taps on 16x16x32;
  // waves (m block of 16 pixels, k step of 32 co) = 4 x 2 ----
  {
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const int mb = wid & 3, kk = wid >> 2;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f}, cor = {0.f, 0.f, 0.f, 0.f};
    const int m = 16 * mb + r16;
    const int win = m >> 2, y = 2 * (win >> 2) + ((m >> 1) & 1), x = 2 * (win & 3) + (m & 1);
    const int abase = y * D2_RS + x * DS_CS + 32 * kk + 8 * kq;
    const int bbase = r16 * WDH_CW + 32 * kk + 8 * kq;
    // 13 steps of a tap pair (2s, 2s + 1): one barrier a pair
    bf16x8 av[2][2][3], bv[2][2][3];
    auto ops = [&](int st, int set) {
      const __bf16* wb = ring2 + (st % 3) * WDHP_SLOT;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = min(2 * st + u, 24);
        const __bf16* pa = D2 + (t / 5) * D2_RS + (t % 5) * DS_CS;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          av[set][u][p] = *reinterpret_cast<const bf16x8*>(pa + p * D2_PL + abase);
          bv[set][u][p] = *reinterpret_cast<const bf16x8*>(wb + u * WDH_SLOT + p * WDH_PL + bbase);
        }
      }
    };
    constexpr int NS = 13;
    ops(0, 0);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      if (st + KD < NS) wd[(st + KD) % KD].load(wt2, wpl, st + KD, half, tid);
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
      if (st + 2 < NS) wd[(st + 2) % KD].store(ring2 + ((st + 2) % 3) * WDHP_SLOT, tid);
      __syncthreads();
    }
    acc += cor;
    DDQ_STAMP(12);
    // the two k steps meet in LDS, summed in order by k step 0
    if (kk == 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) red2[(mb * 4 + e) * 64 + lane] = acc[e];
    }
    __syncthreads();
    float bsum = 0.f;
    if (kk == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += red2[(mb * 4 + e) * 64 + lane];
    }
    __syncthreads();
    for (int f = tid; f < (3 * X1_PL) / 8; f += kThreads) reinterpret_cast<u32x4*>(X)[f] = u32x4{0u, 0u, 0u, 0u};
    if (tid < 484) {   // the frames' halo (fp32 -> bf16 exact), pixel stride 4 bf16
      const int hy = tid / 22, hx = tid - 22 * (tid / 22);
      __bf16 q4[4] = {(__bf16)hv.x, (__bf16)hv.y, (__bf16)hv.z, (__bf16)hv.w};
      *reinterpret_cast<uint2*>(halo + hy * X1_IROW + 4 * hx) = *reinterpret_cast<uint2*>(q4);
    }
    __syncthreads();
    if (kk == 0) {
      // lane: dpool1 at pixels 16 mb + 4 kq + i (window 4 mb + kq of the 8 x 8
      // pool1 grid), channel 16 half + r16 -> pool1's routed quadrant of
      // dconv1, stored at image channel r16 (channels 16..31 stay zero)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int wn = 4 * mb + kq;
        const int y = 2 * (wn >> 2) + (i >> 1), x = 2 * (wn & 3) + (i & 1);
        const int q = m1[(y * 8 + x) * 32 + 16 * half + r16];
        if (q < 4) {
          bsum += acc[i];
          lds_split3(X + ((2 * y + (q >> 1)) * 16 + 2 * x + (q & 1)) * 32 + r16, X1_PL, acc[i]);
        }
      }
    }
    bsm[tid] = bsum;
  }
  __syncthreads();
  DDQ_STAMP(13);

  // ---- conv1's weight gradient (split.h w1_tile_wgrad, one 16-pixel segment
  // per row): wave u < 7 = tap row ky, 16 conv1 rows x 3 MFMAs ----
  {
    const int gq = lane >> 4, iq = (lane & 15) >> 2, ip = lane & 3;
    const int pix0 = 8 * (gq >> 1) + iq;
    const int chn = 16 * (gq & 1) + 4 * ip;
    f32x16 wacc;
#pragma unroll
    for (int e = 0; e < 16; ++e) wacc[e] = 0.f;
    if (wid < 7) {
      const int ky = wid;
      const __bf16* pa0 = X + pix0 * 32 + chn;
      const __bf16* pb0 = halo + ky * X1_IROW + 4 * pix0 + chn;
#pragma unroll 4
      for (int row = 0; row < 16; ++row) {
        bf16x8 av[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const __bf16* pa = pa0 + p * X1_PL + row * 16 * 32;
          av[p] = tr_pair(pa, pa + 4 * 32);
        }
        const __bf16* pb = pb0 + row * X1_IROW;
        const bf16x8 bv = tr_pair(pb, pb + 16);
        wacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv, wacc, 0, 0, 0);
        wacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv, wacc, 0, 0, 0);
        wacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv, wacc, 0, 0, 0);
      }
    }
    __syncthreads();                                  // X / halo reads done
    float* ured = reinterpret_cast<float*>(X);        // [7][16][64]
    if (wid < 7) {
#pragma unroll
      for (int e = 0; e < 16; ++e) ured[(wid * 16 + e) * 64 + lane] = wacc[e];
    }
    __syncthreads();
    // the image's slab, 16-byte write-through stores: item = (ky, row r,
    // half h2, columns 4q..4q+3 < 28); rows co = (r & 3) + 8 (r >> 2) + 4 h2
    const uint32_t slab = (uint32_t)b * 32u * (uint32_t)a.w1_np;
    const __amdgpu_buffer_rsrc_t rs =
        wt_rsrc(a.w1part, (uint32_t)((size_t)B * 32u * (uint32_t)a.w1_np * 4));
    for (int f = tid; f < 7 * 16 * 14; f += kThreads) {
      const int ky = f / 224, rem = f - ky * 224;
      const int r = rem / 14, g = rem - r * 14, h2 = g / 7, q = g - h2 * 7;
      const int co = (r & 3) + 8 * (r >> 2) + 4 * h2;
      if (co >= 16) continue;                         // (the image's zero channels)
      const float4 v = *reinterpret_cast<const float4*>(ured + (ky * 16 + r) * 64 + 32 * h2 + 4 * q);
      wt_store4(rs, (slab + (uint32_t)((16 * half + co) * a.w1_np + ky * 28 + 4 * q)) * 4, v);
    }
    if (tid < 16) {   // bias: channel tid's lanes (r16 = tid) of the k-step-0 waves, in order
      float v = 0.f;
      for (int w = 0; w < 4; ++w)
        for (int g = 0; g < 4; ++g) v += bsm[w * 64 + 16 * g + tid];
      wt_store(rs, (slab + (uint32_t)((16 * half + tid) * a.w1_np + 196)) * 4, v);
    }
  }
  // ---- dconv3 / dconv2 expanded + split, NHWC, out of the images ----
  {
    const int64_t E3 = (int64_t)B * 1024, E2 = (int64_t)B * 4096;
    // (each half writes half of the vectors: channels [32 half, +32))
    for (int f = tid; f < 3 * 16 * 4; f += kThreads) {
      const int p = f / 64, r = f % 64, px = r >> 2, c = 4 * half + (r & 3);
      const u32x4 v = *reinterpret_cast<const u32x4*>(D3 + p * P2_PL + ((px >> 2) + 1) * P2_RS +
                                                       ((px & 3) + 1) * P2_CS + 8 * c);
      *reinterpret_cast<u32x4*>(a.dconv3x + p * E3 + ((size_t)b * 16 + px) * 64 + 8 * c) = v;
    }
    for (int f = tid; f < 3 * 64 * 4; f += kThreads) {
      const int p = f / 256, r = f % 256, px = r >> 2, c = 4 * half + (r & 3);
      const u32x4 v = *reinterpret_cast<const u32x4*>(D2 + p * D2_PL + ((px >> 3) + 2) * D2_RS +
                                                       ((px & 7) + 2) * DS_CS + 8 * c);
      *reinterpret_cast<u32x4*>(a.dconv2x + p * E2 + ((size_t)b * 64 + px) * 64 + 8 * c) = v;
    }
  }
  DDQ_STAMP(14);
}


// ---------------------------------------------------------------------------
// K4: conv2's and conv3's weight gradients, conv1's (the B slabs of K3
// summed), every conv parameter's update, the step's bookkeeping and the next
// step's gather (train_val.prototxt:39-158 weight diffs; server.py apply).
//
// A tile = (layer, tap row ky, block of 32 output channels): 32 co x KS kx x
// CIN ci + 32 biases (ky = 0).  G workgroups per tile each take a group of
// images: the WG stages rounds of images (split dconv rows expanded by K3,
// split input rows of the ky-shifted input, zero halo) into a double buffer,
// its 4 waves split the (image, 16-pixel k step) units of a round, and every
// operand is read transposed out of pixel-major rows (ds_read_b64_tr_b16,
// wgrads.h): 6 MFMAs per (k step, kx, 32 ci).  The waves' tiles meet in LDS
// in fixed order and each WG writes its slab (write-through).  Then the G
// WGs of the tile meet at a counter and each sums a 1/G slice of the tile
// over the G slabs in group order -- the final gradient, updated right there
// (theta, optimizer state, the split layouts, P on a sync step).  No float
// atomics; the sums' order never depends on timing.
// ---------------------------------------------------------------------------
template <int CIN_, int KS_, int HW_>
struct Wg16 {
  static constexpr int CIN = CIN_, KS = KS_, HW = HW_;
  static constexpr int PAD = KS / 2;
  static constexpr int NPX = HW * HW;                 // pixels per image (64 / 16)
  static constexpr int KST = NPX / 16;                // k steps per image (4 / 1)
  static constexpr int NI = 4 / KST;                  // images per round (1 / 4): 4 units
  static constexpr int NCB = CIN / 32;
  static constexpr int NT = KS * NCB;                 // accumulators per wave (5 / 6)
  static constexpr int PSI = CIN == 32 ? 32 : 96;     // input pixel stride (wgrads.h)
  static constexpr int PSD = 32;                      // dconv pixel stride
  static constexpr int SW = HW + 2 * PAD;             // staged input row (halo)
  static constexpr int IN_PL = HW * SW * PSI;         // bf16: HW shifted rows
  static constexpr int D_PL = NPX * PSD;
  static constexpr int IMG = 3 * (IN_PL + D_PL);      // bf16 per staged image
  static constexpr int BUF = NI * IMG;                // bf16 per round buffer
  static constexpr int ELEMS = 32 * KS * CIN;         // [co][kx][ci]
  static constexpr int SLAB = ELEMS + 32;             // + biases
  // vectors (8 channels) a round stages: input, dconv; per thread (256)
  static constexpr int VIN = NI * 3 * HW * HW * (CIN / 8);
  static constexpr int VD = NI * 3 * NPX * 4;
  static constexpr int PIN = (VIN + 255) / 256, PD = (VD + 255) / 256;
  static constexpr int RED = NT * 4 * 16 * 64 * 4 + SLAB * 4;   // the tile sums (wg_tile)
  static constexpr int kSmem = (2 * BUF * 2 > RED ? 2 * BUF * 2 : RED) + 16;
};
using Wg2 = Wg16<32, 5, 8>;
using Wg3 = Wg16<64, 3, 4>;
constexpr int kWgSmem = Wg2::kSmem > Wg3::kSmem ? Wg2::kSmem : Wg3::kSmem;
static_assert(kWgSmem <= 160 * 1024, "K4 LDS");
constexpr int kT2 = 10, kT3 = 6;                      // tiles: 5 ky x 2 co blocks, 3 x 2
constexpr int kW1Blocks = 16;                         // conv1 slab-sum workgroups

struct WgArgs {
  int B;
  int G2, G3, ipg2, ipg3;              // groups per tile, images per group
  const __bf16* pool1s;                // split NHWC (B, 8, 8, 32), plane stride B * 2048
  const __bf16* pool2s;                // split NHWC (B, 4, 4, 64), plane stride B * 1024
  const __bf16* dconv2x;               // split NHWC (B, 8, 8, 64), plane B * 4096 (K3)
  const __bf16* dconv3x;               // split NHWC (B, 4, 4, 64), plane B * 1024 (K3)
  const float* w1part;                 // [B][32][w1_np] (K3)
  int w1_np;
  float* slab2;                        // [10][G2][Wg2::SLAB]
  float* slab3;                        // [6][G3][Wg3::SLAB]
  int32_t* sync;                       // per tile a 64-bit meeting counter (uint64 index
                                       // tile); [32] sticky spin timeout
  float* grad;
  int64_t w_off[3], b_off[3];
  ConvDims cd[3];
  int apply;
  ApplyArgs aa;
  ApplyTail at;
  // bookkeeping (the slab reduce's): apply_book when book
  int book, book_period, book_inc;
  int64_t* iter;
  ReplayMeta* bump;
  Prefetch pf;
  // the fused apply's fc4 weight update (K2 stored the gradient): nw4 blocks
  int64_t w4_off;
  int nw4;
  // B > 32 (K2's G image chunks): the fc4 weight gradient and the unit sums
  // (db4, dW5, db5, loss) summed over the chunks' partials in chunk order
  // here (nw4 blocks, then nus blocks), stored, and applied when apply
  int G, nus;
  const float* upart;
  const float* w4part;
  int64_t b4_off, w5_off, b5_off;
  float* loss;
  // the sticky timeout words of this step's earlier meetings (K2's fan-in,
  // K1's pool2 exchange): set, this launch writes no parameter / state
  const int32_t *poison0, *poison1;
};

// Apply one final conv gradient element (layer l, Caffe index i, local e of
// the layer's weight or bias): grad, and with the fused apply theta / state,
// the split forward layout, P on a sync step.
// th0 / st0: the element's theta and optimizer state, loaded by the caller
// ahead of the sums
__device__ __forceinline__ void conv_final(const WgArgs& a, int l, bool is_w, int64_t i, int e,
                                           float v, float th0, float st0, bool first, bool sync,
                                           bool ap) {
  a.grad[i] = v;
  if (!ap) return;
  float st = (a.aa.rule != 0 && !first) ? st0 : 0.f;
  const float th = apply_rule(a.aa, first, !is_w, th0, v, st);
  a.at.theta[i] = th;
  if (a.aa.rule != 0) a.at.opt[i] = st;
  if (sync) a.at.thetaP[i] = th;
  if (is_w) {
    put_conv_weight(a.cd[l], e, th, a.at.wks, a.at.wks_plane);
    if (sync) put_conv_weight(a.cd[l], e, th, a.at.wksP, a.at.wks_plane);
  }
}

// Element e of a tile's slab (layout [co 32][kx KX][ci CIN], then the 32
// biases of tiles holding tap (ky, kx) = (0, 0)): its Caffe index within the
// layer (le) and flat index (returned); -1 for no element
template <class W, int L, int KX>
__device__ __forceinline__ int64_t tile_elem(const WgArgs& a, int e, int ky, int kx0, int cb,
                                             int& le) {
  constexpr int KS = W::KS, ELEMS = 32 * KX * W::CIN;
  if (e < ELEMS) {
    const int col = e % (KX * W::CIN), co = 32 * cb + e / (KX * W::CIN);
    const int kx = kx0 + col / W::CIN, ci = col % W::CIN;
    le = ((co * W::CIN + ci) * KS + ky) * KS + kx;               // Caffe (co, ci, ky, kx)
    return a.w_off[L] + le;
  }
  le = 0;
  if (ky != 0 || kx0 != 0) return -1;
  le = 32 * cb + e - ELEMS;
  return a.b_off[L] + le;
}

// One weight-gradient tile: output channels [32 cb, +32) x tap row ky x KX
// taps (KX == KS: the whole row; KX == 1: tap kx0 alone), over the images of
// group g.  The rounds' operands are loaded D rounds ahead (a register ring),
// staged through two LDS buffers; the 4 waves' accumulators are summed in
// fixed order in LDS.  G == 1: the tile's sums are final and applied here;
// G > 1: the group's slab, a meeting of the tile's G groups, and this group's
// slice of the tile summed over the slabs in group order and applied.
// ap: the fused apply writes (a.apply, no earlier meeting of the step failed);
// a failed meeting of the tile's groups withholds the slice's writes too.
template <class W, int L, int KX, int D>
__device__ __forceinline__ void wg_tile(const WgArgs& a, char* smem, int tile, int g, int G, int ipg,
                                        float* slabs, bool first, bool sync, bool ap) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int KS = W::KS;
  constexpr int NT = KX * W::NCB;                      // accumulators per wave
  constexpr int ELEMS = 32 * KX * W::CIN, SLAB = ELEMS + 32;
  const int cb = tile & 1;
  const int ky = KX == KS ? tile >> 1 : tile / (2 * KS);
  const int kx0 = KX == KS ? 0 : (tile >> 1) % KS;
  const bool has_bias = ky == 0 && kx0 == 0;
  const int B = a.B;
  const int i0 = g * ipg, i1 = min(B, i0 + ipg);
  const int nimg = max(0, i1 - i0);
  const int nround = (nimg + W::NI - 1) / W::NI;
  __bf16* buf = reinterpret_cast<__bf16*>(smem);
  const __bf16* in = L == 1 ? a.pool1s : a.pool2s;
  const __bf16* dsrc = L == 1 ? a.dconv2x : a.dconv3x;
  const int64_t Ein = (int64_t)B * W::NPX * W::CIN, Ed = (int64_t)B * W::NPX * 64;
  constexpr uint32_t kOOB = 0x80000000u;
  // one descriptor per tensor over its three contiguous planes, the plane in
  // the offset (a descriptor chosen per lane would be a waterfall loop)
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)(3 * Ein * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc((void*)dsrc, (short)0, (int)(3 * Ed * 2), 0x00020000);
  [[maybe_unused]] constexpr int SB = L == 1 ? 24 : 32;   // stamp slots (DDQ_STAMPS builds)
  DDQ_STAMP(SB);
  // the operand ring: round rr in slot rr % D (every index compile-time after
  // unrolling: registers, no scratch)
  u32x4 vin[D][W::PIN], vd[D][W::PD];
  float bsum = 0.f;                                   // has_bias: bias partials (below)
  auto load = [&](int rr, int d) {
#pragma unroll
    for (int u = 0; u < W::PIN; ++u) {
      const int f = tid + 256 * u;
      // f -> (image ii, plane p, row y, px x, chunk c8)
      const int c8 = f % (W::CIN / 8), q1 = f / (W::CIN / 8);
      const int x = q1 % W::HW, q2 = q1 / W::HW, y = q2 % W::HW, q3 = q2 / W::HW;
      const int p = q3 % 3, ii = q3 / 3;
      const int img = i0 + rr * W::NI + ii;
      const int yi = y + ky - W::PAD;
      const bool ok = f < W::VIN && img < i1 && (unsigned)yi < (unsigned)W::HW;
      const uint32_t o = (uint32_t)((p * Ein + ((img * W::HW + yi) * W::HW + x) * W::CIN + 8 * c8) * 2);
      vin[d][u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rin, (int)(ok ? o : kOOB), 0, 0));
    }
#pragma unroll
    for (int u = 0; u < W::PD; ++u) {
      const int f = tid + 256 * u;
      const int c8 = f & 3, q1 = f >> 2;
      const int px = q1 % W::NPX, q2 = q1 / W::NPX, p = q2 % 3, ii = q2 / 3;
      const int img = i0 + rr * W::NI + ii;
      const bool ok = f < W::VD && img < i1;
      const uint32_t o = (uint32_t)((p * Ed + ((img * W::NPX + px) * 64) + 32 * cb + 8 * c8) * 2);
      vd[d][u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, (int)(ok ? o : kOOB), 0, 0));
    }
  };
  // (branch-free: a vector past the round lands in a dummy 16-byte slot after
  // the two buffers -- a store under a branch would make its wait vmcnt(0))
  auto store = [&](int rr, int d) {
    __bf16* bb = buf + (rr & 1) * W::BUF;
    __bf16* dummy = buf + 2 * W::BUF;
#pragma unroll
    for (int u = 0; u < W::PIN; ++u) {
      const int f = tid + 256 * u;
      const int c8 = f % (W::CIN / 8), q1 = f / (W::CIN / 8);
      const int x = q1 % W::HW, q2 = q1 / W::HW, y = q2 % W::HW, q3 = q2 / W::HW;
      const int p = q3 % 3, ii = q3 / 3;
      __bf16* dst = bb + ii * W::IMG + p * W::IN_PL + (y * W::SW + x + W::PAD) * W::PSI + 8 * c8;
      *reinterpret_cast<u32x4*>(f < W::VIN ? dst : dummy) = vin[d][u];
    }
#pragma unroll
    for (int u = 0; u < W::PD; ++u) {
      const int f = tid + 256 * u;
      const int c8 = f & 3, q1 = f >> 2;
      const int px = q1 % W::NPX, q2 = q1 / W::NPX, p = q2 % 3, ii = q2 / 3;
      __bf16* dst = bb + ii * W::IMG + 3 * W::IN_PL + p * W::D_PL + px * W::PSD + 8 * c8;
      *reinterpret_cast<u32x4*>(f < W::VD ? dst : dummy) = vd[d][u];
    }
  };
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int gq = lane >> 4, iq = (lane & 15) >> 2, ip = lane & 3;
  const int pix0 = 8 * (gq >> 1) + iq;                // the lane's pixel of a 16-pixel k step
  const int chn = 16 * (gq & 1) + 4 * ip;
  // unit of wave wid in a round: image ii = wid / KST, k step s = wid % KST
  const int ii = wid / W::KST, s = wid % W::KST;
  // pixels of the lane's two transposed reads (p, p + 4): (y, x) in the map
  const int jA = 16 * s + pix0, jB = jA + 4;
  const int yA = jA / W::HW, xA = jA % W::HW, yB = jB / W::HW, xB = jB % W::HW;
  // (every ring load is issued unconditionally -- rounds past the group read
  // zeros out of range -- so the waits before a round's staging count only
  // the loads issued before its own: a conditional load would force vmcnt(0))
#pragma unroll
  for (int d = 0; d < D; ++d) load(d, d);
  // zero both buffers under the first loads: the input halo columns stay
  // zero (staging writes in-range columns only; out-of-range rows are
  // staged as zero vectors)
  for (int f = tid; f < ((nround > 1 ? 2 : 1) * W::BUF) / 8; f += 256)
    reinterpret_cast<u32x4*>(buf)[f] = u32x4{0u, 0u, 0u, 0u};
  // the direct apply's first elements: theta / state loaded under the rounds
  constexpr int EPD = (SLAB + 255) / 256 < 12 ? (SLAB + 255) / 256 : 12;
  float dth[EPD], dst[EPD];
  {
    const __amdgpu_buffer_rsrc_t rth = __builtin_amdgcn_make_buffer_rsrc(a.at.theta, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t rst = __builtin_amdgcn_make_buffer_rsrc(a.at.opt, (short)0, 0x7fffffff, 0x00020000);
    const bool want = G == 1 && a.apply, wst = want && a.aa.rule != 0;
#pragma unroll
    for (int k = 0; k < EPD; ++k) {   // (unconditional loads, as the ring's)
      int le;
      const int e = tid + 256 * k;
      const int64_t ci = e < SLAB ? tile_elem<W, L, KX>(a, e, ky, kx0, cb, le) : -1;
      dth[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rth, (int)(want && ci >= 0 ? (uint32_t)ci * 4 : kOOB), 0, 0));
      dst[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rst, (int)(wst && ci >= 0 ? (uint32_t)ci * 4 : kOOB), 0, 0));
    }
  }
  __syncthreads();
  for (int r0 = 0; r0 < nround; r0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int rr = r0 + d;
      if (rr >= nround) break;
      store(rr, d);
      __syncthreads();                                // round rr staged; round rr - 1 computed
      if (rr == 0) DDQ_STAMP(SB + 1);
      load(rr + D, d);
      __builtin_amdgcn_sched_barrier(0);
      const int img = i0 + rr * W::NI + ii;
      if (img < i1) {
        const __bf16* bb = buf + (rr & 1) * W::BUF + ii * W::IMG;
        bf16x8 av[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const __bf16* pa = bb + 3 * W::IN_PL + p * W::D_PL + chn;
          av[p] = tr_pair(pa + jA * W::PSD, pa + jB * W::PSD);
        }
#pragma unroll
        for (int kk = 0; kk < KX; ++kk) {
          const int kx = kx0 + kk;
#pragma unroll
          for (int c = 0; c < W::NCB; ++c) {
            bf16x8 bv[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              const __bf16* pb = bb + p * W::IN_PL + 32 * c + chn;
              bv[p] = tr_pair(pb + (yA * W::SW + xA + kx) * W::PSI, pb + (yB * W::SW + xB + kx) * W::PSI);
            }
            const int t = kk * W::NCB + c;
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv[0], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[1], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[2], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[0], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[1], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[0], acc[t], 0, 0, 0);
          }
        }
      }
      if (has_bias) {
        // bias partial: thread = (channel c = tid & 31, pixel slice tid >> 5)
        // over the round's 64 staged dconv pixels, the fp32 value of a split
        // element being the sum of its planes
        const __bf16* bb = buf + (rr & 1) * W::BUF;
        const int c = tid & 31;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int q = 8 * (tid >> 5) + k;               // pixel q of the round (NI images)
          const int iq2 = q / W::NPX, px = q % W::NPX;
          if (i0 + rr * W::NI + iq2 < i1) {
            const __bf16* pd = bb + iq2 * W::IMG + 3 * W::IN_PL + px * W::PSD + c;
            bsum += ((float)pd[0] + (float)pd[W::D_PL]) + (float)pd[2 * W::D_PL];
          }
        }
      }
      __syncthreads();                                // round rr's reads done (its buffer is reused)
    }
  }
  if (has_bias) {   // the 8 pixel slices of each channel, in order
    float* bred = reinterpret_cast<float*>(smem);
    bred[tid] = bsum;
    __syncthreads();
    if (tid < 32) {
      float v = bred[tid];
#pragma unroll
      for (int k = 1; k < 8; ++k) v += bred[32 * k + tid];
      bsum = v;
    }
  }
  DDQ_STAMP(SB + 2);
  // ---- the waves' tiles summed in fixed order -> LDS (G == 1) or the slab:
  // every accumulator of every wave into LDS at once (the staging buffers are
  // dead), one barrier, then each thread's 4-wave sums of all NT tiles ----
  float* red = reinterpret_cast<float*>(smem);        // [NT][4 waves][16][64]
  float* fin = red + NT * 4 * 16 * 64;                // G == 1: the tile's sums [SLAB]
  float* slab = slabs + ((int64_t)tile * G + g) * SLAB;
  const __amdgpu_buffer_rsrc_t srs = wt_rsrc(slab, (uint32_t)(SLAB * 4));
  __syncthreads();                                    // (bias slice sums read above)
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((t * 4 + wid) * 16 + r) * 64 + lane] = acc[t][r];
  __syncthreads();
  {   // thread = (tile row r, lanes 4q..4q+3)
    const int r = tid >> 4, l0 = 4 * (tid & 15);
    const int e = r * 64 + l0;
    const int co = (r & 3) + 8 * (r >> 2) + 4 * (l0 >> 5);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float* rt = red + t * 4096 + e;
      const float4 a0 = *reinterpret_cast<const float4*>(rt);
      const float4 a1 = *reinterpret_cast<const float4*>(rt + 1024);
      const float4 a2 = *reinterpret_cast<const float4*>(rt + 2048);
      const float4 a3 = *reinterpret_cast<const float4*>(rt + 3072);
      const float4 v = make_float4((a0.x + a1.x) + (a2.x + a3.x), (a0.y + a1.y) + (a2.y + a3.y),
                                   (a0.z + a1.z) + (a2.z + a3.z), (a0.w + a1.w) + (a2.w + a3.w));
      const int kk = t / W::NCB, c = t % W::NCB;
      const int o = (co * KX + kk) * W::CIN + 32 * c + (l0 & 31);
      if (G == 1) *reinterpret_cast<float4*>(fin + o) = v;
      else wt_store4(srs, (uint32_t)(o * 4), v);
    }
  }
  if (G == 1) {
    if (tid < 32) fin[ELEMS + tid] = has_bias ? bsum : 0.f;
    __syncthreads();
    DDQ_STAMP(SB + 3);
    DDQ_STAMP(SB + 4);
    for (int c0 = 0; c0 < SLAB; c0 += 256 * EPD) {
#pragma unroll
      for (int k = 0; k < EPD; ++k) {
        const int e = c0 + tid + 256 * k;
        if (e >= SLAB) continue;
        int le;
        const int64_t ci = tile_elem<W, L, KX>(a, e, ky, kx0, cb, le);
        if (ci < 0) continue;
        float th = dth[k], st = dst[k];
        if (c0 > 0 && a.apply) {                      // past the preloaded chunk
          th = a.at.theta[ci];
          st = a.aa.rule != 0 ? a.at.opt[ci] : 0.f;
        }
        conv_final(a, L, e < ELEMS, ci, le, fin[e], th, st, first, sync, ap);
      }
    }
    DDQ_STAMP(SB + 5);
    return;
  }
  if (tid < 32) wt_store(srs, (uint32_t)((ELEMS + tid) * 4), has_bias ? bsum : 0.f);
  // ---- meet the tile's other groups, then sum and update a slice ----
  // the slice this workgroup finishes: its elements' Caffe index, theta and
  // optimizer state loaded before the meeting (they do not depend on it)
  const int sl = (SLAB + G - 1) / G, e0 = g * sl, e1 = min(SLAB, e0 + sl);
  constexpr int EPT = 8;                              // elements a thread per chunk (one chunk
  uint64_t* ctr = reinterpret_cast<uint64_t*>(a.sync) + (L == 1 ? 0 : kT2) + tile;   // at G >= 4)
  const __amdgpu_buffer_rsrc_t rall = __builtin_amdgcn_make_buffer_rsrc(
      slabs + (int64_t)tile * G * SLAB, (short)0, (int)(G * SLAB * 4), 0x00020000);
  if (e0 >= e1) meet(ctr, G, a.sync + 32);            // an empty slice still arrives
  int32_t mword = 0;
  for (int c0 = e0; c0 < e1; c0 += 256 * EPT) {
    int64_t ci_[EPT];
    int le_[EPT];
    float th_[EPT], st_[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = c0 + tid + 256 * k;
      ci_[k] = -1; le_[k] = 0; th_[k] = 0.f; st_[k] = 0.f;
      if (e >= e1) continue;
      ci_[k] = tile_elem<W, L, KX>(a, e, ky, kx0, cb, le_[k]);
      if (ci_[k] >= 0 && a.apply) {
        th_[k] = a.at.theta[ci_[k]];
        if (a.aa.rule != 0) st_[k] = a.at.opt[ci_[k]];
      }
    }
    if (c0 == e0) {
      DDQ_STAMP(SB + 3);
      meet(ctr, G, a.sync + 32);
      if (ap) mword = meet_word(a.sync + 32);           // (consumed at the updates)
      DDQ_STAMP(SB + 4);
    }
    // every group's value of every element loaded first (G <= GM), summed in
    // group order, then the stores
    constexpr int GM = L == 1 ? 16 : 8;
    float vs[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = c0 + tid + 256 * k;
      vs[k] = 0.f;
      if (c0 + 256 * k >= e1) continue;                // (wave-uniform: no element left)
      float t[GM];
#pragma unroll
      for (int gg = 0; gg < GM; ++gg)
        t[gg] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rall, (int)(gg < G && e < e1 ? (gg * SLAB + e) * 4 : 0x80000000u), 0, 16));
      float v = t[0];
#pragma unroll
      for (int gg = 1; gg < GM; ++gg)
        if (gg < G) v += t[gg];
      vs[k] = v;
    }
#ifdef DDQ_STAMPS
    if (c0 == e0) {   // (phase stamps: the sums landed)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      DDQ_STAMP(SB + 6);
    }
#endif
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      const int e = c0 + tid + 256 * k;
      if (e < e1 && ci_[k] >= 0)
        conv_final(a, L, e < ELEMS, ci_[k], le_[k], vs[k], th_[k], st_[k], first, sync, ap && mword == 0);
    }
  }
  DDQ_STAMP(SB + 5);
}

// fc4's weights (512 x 256 at S = 16) updated from the gradient K2 stored, 4
// consecutive elements a thread (coalesced), the rules of the other apply
// sites (apply_rule, no FMA contraction: bit-identical updates)
__device__ __forceinline__ void w4_apply(const WgArgs& a, int blk, bool first, bool sync, bool ap) {
  constexpr int64_t n = 512LL * kFcK;
  if (a.G == 1 && !ap) return;
  for (int64_t j = ((int64_t)blk * 256 + threadIdx.x) * 4; j < n; j += (int64_t)a.nw4 * 256 * 4) {
    const int64_t i = a.w4_off + j;
    float4 g;
    if (a.G > 1) {   // the chunks' partials in chunk order -> the gradient
      g = *reinterpret_cast<const float4*>(a.w4part + j);
      for (int cc = 1; cc < a.G; ++cc) {
        const float4 p = *reinterpret_cast<const float4*>(a.w4part + (int64_t)cc * n + j);
        g.x += p.x; g.y += p.y; g.z += p.z; g.w += p.w;
      }
      *reinterpret_cast<float4*>(a.grad + i) = g;
      if (!ap) continue;
    } else {
      g = *reinterpret_cast<const float4*>(a.grad + i);
    }
    const float4 t = *reinterpret_cast<const float4*>(a.at.theta + i);
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.aa.rule != 0 && !first) o = *reinterpret_cast<const float4*>(a.at.opt + i);
    const float gg[4] = {g.x, g.y, g.z, g.w};
    float th[4] = {t.x, t.y, t.z, t.w}, st[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) th[e] = apply_rule(a.aa, first, false, th[e], gg[e], st[e]);
    const float4 t4 = make_float4(th[0], th[1], th[2], th[3]);
    *reinterpret_cast<float4*>(a.at.theta + i) = t4;
    if (a.aa.rule != 0) *reinterpret_cast<float4*>(a.at.opt + i) = make_float4(st[0], st[1], st[2], st[3]);
    if (sync) *reinterpret_cast<float4*>(a.at.thetaP + i) = t4;
  }
}

// B <= 32: Q_out's biases from the gradient K2 stored (K2 leaves their update
// here: every K2 workgroup reads them after its fan-in)
__device__ __forceinline__ void b5_apply(const WgArgs& a, bool first, bool sync, bool ap) {
  const int t = threadIdx.x;
  if (!ap || t >= 4) return;
  const int64_t i = a.b5_off + t;
  const float v = a.grad[i];
  float st = (a.aa.rule != 0 && !first) ? a.at.opt[i] : 0.f;
  const float th = apply_rule(a.aa, first, true, a.at.theta[i], v, st);
  a.at.theta[i] = th;
  if (a.aa.rule != 0) a.at.opt[i] = st;
  if (sync) a.at.thetaP[i] = th;
}

// B > 32: the unit sums' partials (K2 upart) summed in chunk order -> db4,
// dW5 (32 blocks x 80), db5 (4), loss; stored, and applied when apply
__device__ __forceinline__ void units_apply(const WgArgs& a, bool first, bool sync, bool ap) {
  for (int q = threadIdx.x; q < kFcBlk * 85; q += 256) {
    const int jb = q / 85, qq = q - jb * 85;
    if (qq >= 80 && jb != 0) continue;                // (db5, loss: block 0's)
    float v = a.upart[jb * 96 + qq];
    for (int cc = 1; cc < a.G; ++cc) v += a.upart[(cc * kFcBlk + jb) * 96 + qq];
    if (qq == 84) { *a.loss = v / (float)a.B / 2.f; continue; }
    const int n0 = jb * kFcN;
    const int64_t i = qq >= 80 ? a.b5_off + (qq - 80)
                               : ((qq >> 4) == 0 ? a.b4_off + n0 + (qq & 15)
                                                 : a.w5_off + ((qq >> 4) - 1) * 512 + n0 + (qq & 15));
    const bool is_bias = qq >= 80 || (qq >> 4) == 0;
    a.grad[i] = v;
    if (!ap) continue;
    float st = (a.aa.rule != 0 && !first) ? a.at.opt[i] : 0.f;
    const float th = apply_rule(a.aa, first, is_bias, a.at.theta[i], v, st);
    a.at.theta[i] = th;
    if (a.aa.rule != 0) a.at.opt[i] = st;
    if (sync) a.at.thetaP[i] = th;
  }
}

// Block order: conv3's tiles (the longest chains) first, conv2's, then
// conv1's slab sums and the next step's gather (short, no meeting) -- every
// meeting workgroup is dispatched before any block that could hold a CU.
__global__ __launch_bounds__(256) void wgrad16_kernel(const WgArgs a) {
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  int bid = blockIdx.x;
  const bool first = a.apply && a.at.opt_init[2] != 0, sync = a.apply && a.at.opt_init[3] != 0;
  // (read now, needed only at the writes: the operand loads do not wait on it)
  const bool pois = a.apply && step_poisoned(a.poison0, a.poison1);
  const bool ap = a.apply && !pois;
  const int n2 = kT2 * a.G2, n3 = kT3 * a.G3;
  if (bid < n3) {
    wg_tile<Wg3, 2, 3, 2>(a, wsm, bid % kT3, bid / kT3, a.G3, a.ipg3, a.slab3, first, sync, ap);
    return;
  }
  bid -= n3;
  if (bid < n2) {
    wg_tile<Wg2, 1, 5, 2>(a, wsm, bid % kT2, bid / kT2, a.G2, a.ipg2, a.slab2, first, sync, ap);
    return;
  }
  bid -= n2;
  if (bid >= kW1Blocks) {   // the fc4 weights' (and unit sums') update, then the next
    const int x = bid - kW1Blocks;   // step's gather (B = 256: 512 short blocks, last)
    if (x < a.nw4) {
      w4_apply(a, x, first, sync, ap);
      if (x == 0 && a.G == 1) b5_apply(a, first, sync, ap);
    }
    else if (x < a.nw4 + a.nus) units_apply(a, first, sync, ap);
    else prefetch_body(a.pf, x - a.nw4 - a.nus);
    return;
  }
  DDQ_STAMP(40);
  // conv1: the B per-image slabs summed in image order, element by element
  if (bid == 0 && threadIdx.x == 0 && a.book && !pois)   // (no update: no iteration)
    apply_book(a.iter, const_cast<int32_t*>(a.at.opt_init), a.book_period, a.bump, a.book_inc);
  const int np = a.w1_np;
  for (int e = bid * 256 + threadIdx.x; e < 32 * 197; e += kW1Blocks * 256) {
    const int co = e / 197, n = e - co * 197;
    int le;
    int64_t i;
    if (n < 196) {
      const int ky = n / 28, kx = (n % 28) >> 2, ci = n & 3;
      le = ((co * 4 + ci) * 7 + ky) * 7 + kx;                    // Caffe (co, ci, ky, kx)
      i = a.w_off[0] + le;
    } else {
      le = co;
      i = a.b_off[0] + co;
    }
    float th0 = 0.f, st0 = 0.f;                                   // ahead of the slab loads
    if (a.apply) {
      th0 = a.at.theta[i];
      if (a.aa.rule != 0) st0 = a.at.opt[i];
    }
    const float* src = a.w1part + co * np + n;
    float v = 0.f;
    int b0 = 0;
    for (; b0 + 32 <= a.B; b0 += 32) {   // 32 loads in flight a round (B = 256: 8 rounds)
      float t[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) t[u] = src[(int64_t)(b0 + u) * 32 * np];
#pragma unroll
      for (int u = 0; u < 32; ++u) v += t[u];
    }
    for (; b0 + 8 <= a.B; b0 += 8) {
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = src[(int64_t)(b0 + u) * 32 * np];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += t[u];
    }
    for (; b0 < a.B; ++b0) v += src[(int64_t)b0 * 32 * np];
    conv_final(a, 0, n < 196, i, le, v, th0, st0, first, sync, ap);
  }
  DDQ_STAMP(41);
}

}  // namespace sm16
}  // namespace ddq
