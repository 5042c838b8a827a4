// deepq step kernels for MI355X (gfx950).  See DESIGN.md for the data layout
// and the roofline of each kernel.
#include "kernels.h"
#include "wgrads.h"
#include "fc.h"
#include "split.h"
#include "small.h"

namespace ddq {

// first failing launch site of the last failed launch sequence (api.hip
// appends it to the error message)
thread_local const char* g_launch_where = "";
thread_local ExtTiming g_ext_timing;
thread_local bool g_profiling = false;
thread_local int g_unmarked = 0;
#ifdef DDQ_STAMPS
__device__ uint64_t g_stamps[kStampBlocks * kStampSlots];
}  // namespace ddq
// variant builds only (common.h DDQ_STAMP): copy the stamp table out, then
// clear it.  0 = ok, -1 = size mismatch, -3 = HIP error (ddq_hip.h codes)
extern "C" int ddq_debug_stamps(uint64_t* out, int64_t n) {
  using namespace ddq;
  const size_t bytes = sizeof(uint64_t) * kStampBlocks * kStampSlots;
  if (n * (int64_t)sizeof(uint64_t) != (int64_t)bytes) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), bytes) != hipSuccess) return -3;
  static uint64_t zeros[kStampBlocks * kStampSlots];
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zeros, bytes) != hipSuccess) return -3;
  return 0;
}
namespace ddq {
#endif
#define DDQ_STR2(x) #x
#define DDQ_STR(x) DDQ_STR2(x)
#define CHECK_LAUNCH(x)                                             \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      if (!*g_launch_where) g_launch_where = "kernels.hip:" DDQ_STR(__LINE__); \
      return e_;                                                    \
    }                                                               \
  } while (0)

// ---------------------------------------------------------------------------
// layout
// ---------------------------------------------------------------------------
ParamLayout make_layout(int S) {
  ParamLayout L;
  L.S = S; L.S2 = S / 2; L.S3 = S / 4; L.S4 = S / 8;
  const int64_t k4 = 64ll * L.S4 * L.S4;
  const int64_t wn[5] = {32ll * 4 * 49, 64ll * 32 * 25, 64ll * 64 * 9, 512ll * k4, 4ll * 512};
  const int64_t bn[5] = {32, 64, 64, 512, 4};
  int64_t o = 0;
  for (int i = 0; i < 5; ++i) {
    L.w[i] = o; L.wn[i] = wn[i]; o += wn[i];
    L.b[i] = o; L.bn[i] = bn[i]; o += bn[i];
  }
  L.total = o;
  // split forward weights: conv1 [n][7][8][4] (kx 7 zero), conv2/3 [co][tap][ci]
  L.wks_off[0] = 0;
  L.wks_off[1] = kConv1WPlane;
  L.wks_off[2] = L.wks_off[1] + wn[1];
  // the conv2 data gradient's weights: Q's split conv2 weights transposed and
  // flipped, Wt[ci][tap'][co] = W[co][ci][4-ky][4-kx] (rebuilt by the head
  // kernel of every step from the forward layout)
  L.wkst_off = L.wks_off[2] + wn[2];
  L.wkst3_off = L.wkst_off + wn[1];   // conv3's likewise (Wt[ci][8-tap][co])
  L.wks_total = L.wkst3_off + wn[2];
  return L;
}

double step_flops(int B, int S) {
  // F = B*(6272 S1^2 + 51200 S2^2 + 36864 S3^2 + 32768 S4^2 + 2048)
  // MACs per tower forward; step = Q fwd + P fwd + Q wgrad + Q dgrad (no conv1 dgrad).
  const double s1 = S, s2 = S / 2, s3 = S / 4, s4 = S / 8;
  const double F = (double)B * (6272 * s1 * s1 + 51200 * s2 * s2 + 36864 * s3 * s3 +
                                32768 * s4 * s4 + 2048);
  return 2.0 * (4 * F - 6272.0 * B * s1 * s1);
}

// ---------------------------------------------------------------------------
// replay: index draw (device RNG) and minibatch gather (replay.py:144-183)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// One workgroup: B <= blockDim distinct indices, uniform over [0,valid) \ {head-1}
// (the distribution of replay.py:152-157's whole-list redraw), sorted into
// cand[0..B).  Colliding / forbidden draws are redrawn independently each
// round; the process is symmetric in the population, so the final set is
// uniform.  Deterministic in (seed, ctr): every workgroup that runs it gets
// the same set, which lets the gather workgroups draw for themselves.
constexpr int kDrawRounds = 4096;

__device__ void draw_sorted(ReplayMeta* meta, int B, uint64_t seed, uint64_t ctr,
                            int64_t* cand, int* bad_any) {
  const int t = threadIdx.x;
  const int64_t valid = meta->valid;
  const int64_t forbid = meta->head - 1;   // -1 when head == 0: nothing forbidden
  // draw for sorted position `pos` in redraw round `round`
  auto draw_at = [&](int round, int pos) -> int64_t {
    uint64_t r = splitmix64(seed ^ splitmix64(ctr * 0x100000001B3ull + (uint64_t)pos * 0x9E37ull +
                                              ((uint64_t)round << 40)));
    return (int64_t)__umul64hi(r, (uint64_t)valid);
  };
  auto draw = [&](int round) -> int64_t { return draw_at(round, t); };
  if (B <= 64) {
    // One wave, no sort network: lane t keeps its draw and computes its
    // sorted position by comparing against every lane (readlane, no LDS
    // round trips -- the 21-stage shuffle bitonic sort it replaces was a
    // chain of ds_bpermute latencies).  Ties rank by lane, so the positions
    // a duplicate group occupies are the bitonic path's; the later ones are
    // redrawn with their position as hash input, exactly as there (and as
    // the multi-wave path below), so the sorted set is unchanged.  Indices
    // fit 32 bits (valid < 2^31); head-1 = -1 never matches a draw.
    if (t < 64) {
      uint32_t v = (t < B) ? (uint32_t)draw_at(0, t) : 0xFFFFFFFFu;
      const uint32_t fb = (uint32_t)forbid;
      int r = t;
      bool done = false;
      for (int round = 1; round <= kDrawRounds; ++round) {
        int less = 0, eqlo = 0;
        for (int k = 0; k < B; ++k) {
          const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)v, k);
          less += o < v;
          eqlo += (o == v) & (k < t);
        }
        r = less + eqlo;
        const bool bad = t < B && (v == fb || eqlo > 0);
        if (__ballot(bad) == 0) { done = true; break; }
        if (round < kDrawRounds && bad) v = (uint32_t)draw_at(round, r);
      }
      // no distinct set after kDrawRounds checked rounds (valid barely above
      // B): flag it (ddq_replay_status) instead of gathering a bad set silently
      if (!done && t == 0) meta->err = 2;
      if (t < B) cand[r] = (int64_t)v;
    }
    __syncthreads();
    return;
  }
  int P2 = 1;
  while (P2 < B) P2 <<= 1;
  if (t < P2) cand[t] = (t < B) ? draw(0) : INT64_MAX;
  for (int round = 1; round <= kDrawRounds; ++round) {
    __syncthreads();
    // bitonic sort of cand[0..P2)
    for (int k = 2; k <= P2; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        if (t < P2) {
          const int p = t ^ j;
          if (p > t) {
            const bool up = (t & k) == 0;
            const int64_t a = cand[t], b = cand[p];
            if ((a > b) == up) { cand[t] = b; cand[p] = a; }
          }
        }
        __syncthreads();
      }
    }
    if (t == 0) *bad_any = 0;
    __syncthreads();
    bool bad = false;
    if (t < B) bad = (cand[t] == forbid) || (t > 0 && cand[t] == cand[t - 1]);
    if (bad) *bad_any = 1;
    __syncthreads();
    if (!*bad_any) break;
    if (round == kDrawRounds) {   // checked and still bad: flag it (see above)
      if (t == 0) meta->err = 2;
      break;
    }
    if (bad) cand[t] = draw(round);
  }
  __syncthreads();
}

// Index log (ddq_index_log_enable): draw `ctr`'s sorted set, B entries.
__device__ __forceinline__ void log_draw(int32_t* log, int64_t cap, uint64_t ctr, int B, int t,
                                         int32_t v) {
  if (log && t < B) log[(int64_t)(ctr % (uint64_t)cap) * B + t] = v;
}

__global__ __launch_bounds__(1024) void sample_kernel(ReplayMeta* meta, int B, uint64_t seed,
                                                      int32_t* idx_out, int32_t* log,
                                                      int64_t log_cap) {
  __shared__ int64_t cand[1024];
  __shared__ int bad_any;
  const uint64_t ctr = meta->counter;
  draw_sorted(meta, B, seed, ctr, cand, &bad_any);
  const int t = threadIdx.x;
  if (t < B) idx_out[t] = (int32_t)cand[t];
  log_draw(log, log_cap, ctr, B, t, (int32_t)cand[t < B ? t : 0]);
  if (t == 0) meta->counter = ctr + 1;
}

// u8 (C,H,W) slot -> f32 NHWC, 4 pixels per thread; z = 0 -> state from
// idx, z = 1 -> next_state from next_idx (wrap N-1 -> 0, replay.py:160-166);
// the z = 1 blocks with blockIdx.x == 0 also write action one-hot, reward and
// non_terminal of next_idx (replay.py:172-183).
__device__ __forceinline__ void gather_body(
    const uint8_t* __restrict__ st, const uint8_t* __restrict__ act,
    const int16_t* __restrict__ rew, const uint8_t* __restrict__ nt, ReplayMeta* meta, int64_t i,
    int S, float* __restrict__ sQ, float* __restrict__ sP, float* __restrict__ action,
    float* __restrict__ reward, float* __restrict__ nonterm, int bx, int b, int z) {
  const int64_t N = meta->capacity;
  const int64_t nxt = (i + 1 == N) ? 0 : i + 1;
  const int64_t slot = z ? nxt : i;
  const int SS = S * S;
  const int p4 = bx * 256 + threadIdx.x;             // group of 4 pixels
  if (p4 * 4 < SS) {
    const uint8_t* src = st + slot * 4 * SS + p4 * 4;
    const uchar4 c0 = *reinterpret_cast<const uchar4*>(src);
    const uchar4 c1 = *reinterpret_cast<const uchar4*>(src + SS);
    const uchar4 c2 = *reinterpret_cast<const uchar4*>(src + 2 * SS);
    const uchar4 c3 = *reinterpret_cast<const uchar4*>(src + 3 * SS);
    float4* dst = reinterpret_cast<float4*>((z ? sP : sQ) + ((size_t)b * SS + p4 * 4) * 4);
    dst[0] = f4(c0.x, c1.x, c2.x, c3.x);
    dst[1] = f4(c0.y, c1.y, c2.y, c3.y);
    dst[2] = f4(c0.z, c1.z, c2.z, c3.z);
    dst[3] = f4(c0.w, c1.w, c2.w, c3.w);
  }
  if (z == 1 && bx == 0 && threadIdx.x < 4) {
    const int a = act[nxt];
    if (a >= kActions) meta->err = 1;
    action[b * 4 + threadIdx.x] = (threadIdx.x == a) ? 1.f : 0.f;
    if (threadIdx.x == 0) {
      reward[b] = (float)rew[nxt];
      nonterm[b] = nt[nxt] ? 1.f : 0.f;
    }
  }
}

// grid (ceil(S*S/4/256), B, 2), indices from idx (host draw or sample_kernel)
__global__ __launch_bounds__(256) void gather_kernel(
    const uint8_t* __restrict__ st, const uint8_t* __restrict__ act,
    const int16_t* __restrict__ rew, const uint8_t* __restrict__ nt, ReplayMeta* meta,
    const int32_t* __restrict__ idx, int S, float* __restrict__ sQ, float* __restrict__ sP,
    float* __restrict__ action, float* __restrict__ reward, float* __restrict__ nonterm) {
  gather_body(st, act, rew, nt, meta, idx[blockIdx.y], S, sQ, sP, action, reward, nonterm,
              blockIdx.x, blockIdx.y, blockIdx.z);
}

// Fused draw + gather for the training step (B <= 256): every workgroup
// draws the same sorted index set (draw_sorted) and gathers its own sample.
// The device counter is NOT advanced here (every workgroup must read the
// same value); the step's apply bookkeeping advances it.
__global__ __launch_bounds__(256) void sample_gather_kernel(
    const uint8_t* __restrict__ st, const uint8_t* __restrict__ act,
    const int16_t* __restrict__ rew, const uint8_t* __restrict__ nt, ReplayMeta* meta, int B,
    uint64_t seed, int32_t* __restrict__ idx_out, int S, float* __restrict__ sQ,
    float* __restrict__ sP, float* __restrict__ action, float* __restrict__ reward,
    float* __restrict__ nonterm, int32_t* log, int64_t log_cap) {
  __shared__ int64_t cand[256];
  __shared__ int bad_any;
  const uint64_t ctr = meta->counter;
  draw_sorted(meta, B, seed, ctr, cand, &bad_any);
  if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x < B) {
    idx_out[threadIdx.x] = (int32_t)cand[threadIdx.x];
    log_draw(log, log_cap, ctr, B, threadIdx.x, (int32_t)cand[threadIdx.x]);
  }
  gather_body(st, act, rew, nt, meta, cand[blockIdx.y], S, sQ, sP, action, reward, nonterm,
              blockIdx.x, blockIdx.y, blockIdx.z);
}

hipError_t launch_sample(const NetBuffers& nb, ReplayMeta* meta, uint64_t seed, hipStream_t s) {
  int threads = 64;                 // one wave for B <= 64: cheap barriers
  while (threads < nb.B) threads <<= 1;
  ddq_launch(sample_kernel, dim3(1), dim3(threads), 0, s, meta, nb.B, seed, nb.idx,
                     nb.idx_log, nb.log_cap);
  return hipGetLastError();
}

hipError_t launch_sample_gather(const NetBuffers& nb, const uint8_t* st, const uint8_t* act,
                                const int16_t* rew, const uint8_t* nt, ReplayMeta* meta,
                                uint64_t seed, hipStream_t s) {
  const int SS = nb.S * nb.S;
  dim3 grid((SS / 4 + 255) / 256, nb.B, 2);
  ddq_launch(sample_gather_kernel, grid, dim3(256), 0, s, st, act, rew, nt, meta, nb.B,
                     seed, nb.idx, nb.S, nb.state, nb.next_state, nb.action, nb.reward,
                     nb.nonterm, nb.idx_log, nb.log_cap);
  return hipGetLastError();
}

hipError_t launch_gather(const NetBuffers& nb, const uint8_t* st, const uint8_t* act,
                         const int16_t* rew, const uint8_t* nt, ReplayMeta* meta,
                         hipStream_t s) {
  const int SS = nb.S * nb.S;
  dim3 grid((SS / 4 + 255) / 256, nb.B, 2);
  ddq_launch(gather_kernel, grid, dim3(256), 0, s, st, act, rew, nt, meta, nb.idx, nb.S,
                     nb.state, nb.next_state, nb.action, nb.reward, nb.nonterm);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// large-batch sampling + Caffe-layout gather (SURVEY 8(d) C5 gather stress;
// same selection semantics as replay.py:144-183 for any n <= valid/2)
// ---------------------------------------------------------------------------
// Claim: thread t draws uniform x in [0,valid) until it sets a fresh bit of
// the bitmap (head-1 never accepted).  Every draw sequence is i.i.d. and the
// process is symmetric in the population, so the claimed set is a uniform
// n-subset of [0,valid) \ {head-1} -- the distribution of the reference's
// whole-list redraw.  The bitmap is then compacted in index order, which is
// the sort of replay.py:159 for free.
__global__ __launch_bounds__(256) void claim_kernel(ReplayMeta* meta, int n, uint64_t seed,
                                                   uint64_t ctr, uint32_t* __restrict__ bm) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const int64_t valid = meta->valid, forbid = meta->head - 1;
  for (int round = 0; round < 4096; ++round) {
    const uint64_t r = splitmix64(seed ^ splitmix64(ctr * 0x100000001B3ull +
                                                    (uint64_t)t * 0x9E3779B1ull +
                                                    ((uint64_t)round << 44)));
    const int64_t x = (int64_t)__umul64hi(r, (uint64_t)valid);
    if (x == forbid) continue;
    const uint32_t bit = 1u << (x & 31);
    if (!(atomicOr(&bm[x >> 5], bit) & bit)) return;
  }
  meta->err = 2;   // n too close to valid (cannot happen for n <= valid/2 in practice)
}

// inclusive scan of v over the 256-thread workgroup; returns the exclusive
// prefix and writes the workgroup total to *tot
__device__ __forceinline__ int block_scan_256(int v, int* tot) {
  __shared__ int wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += wsum[i];
  *tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return base + x - v;
}

// 4 bitmap words per thread, 1024 per workgroup
__device__ __forceinline__ uint4 bm_words(const uint32_t* bm, int64_t nwords, int64_t w0) {
  uint4 q = make_uint4(0, 0, 0, 0);
  if (w0 + 3 < nwords) {
    q = *reinterpret_cast<const uint4*>(bm + w0);
  } else {
    if (w0 < nwords) q.x = bm[w0];
    if (w0 + 1 < nwords) q.y = bm[w0 + 1];
    if (w0 + 2 < nwords) q.z = bm[w0 + 2];
  }
  return q;
}

__global__ __launch_bounds__(256) void bm_count_kernel(const uint32_t* __restrict__ bm,
                                                       int64_t nwords, int32_t* __restrict__ tot) {
  const int64_t w0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const uint4 q = bm_words(bm, nwords, w0);
  const int c = __popc(q.x) + __popc(q.y) + __popc(q.z) + __popc(q.w);
  int t;
  block_scan_256(c, &t);
  if (threadIdx.x == 0) tot[blockIdx.x] = t;
}

// exclusive scan of the per-workgroup counts (one workgroup, any length)
__global__ __launch_bounds__(256) void bm_scan_kernel(int32_t* __restrict__ tot, int nblk) {
  int carry = 0;
  for (int b0 = 0; b0 < nblk; b0 += 256) {
    const int i = b0 + threadIdx.x;
    const int v = i < nblk ? tot[i] : 0;
    int t;
    const int ex = block_scan_256(v, &t);
    if (i < nblk) tot[i] = carry + ex;
    carry += t;
  }
}

__global__ __launch_bounds__(256) void bm_emit_kernel(const uint32_t* __restrict__ bm,
                                                      int64_t nwords,
                                                      const int32_t* __restrict__ off,
                                                      int32_t* __restrict__ idx, int n) {
  const int64_t w0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const uint4 q = bm_words(bm, nwords, w0);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
  int t;
  int pos = off[blockIdx.x] +
            block_scan_256(__popc(w[0]) + __popc(w[1]) + __popc(w[2]) + __popc(w[3]), &t);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v = w[k];
    while (v) {
      const int b = __ffs(v) - 1;
      if (pos < n) idx[pos] = (int32_t)((w0 + k) * 32 + b);
      ++pos;
      v &= v - 1;
    }
  }
}

// u8 (C,H,W) slots -> f32 Caffe (n,4,S,S).  blockIdx.x = (row b, slice):
// a row's wps 4-byte words are cut into cpr slices of 512, so the slot index
// is one uniform load a workgroup (no per-lane divide, no per-lane index
// load ahead of the data load).  Each thread: 2 dword loads at stride 256
// (a wave instruction reads 256 contiguous bytes), then 2 float4
// non-temporal stores (a wave instruction writes 1 KiB contiguous).  Against
// the round-4 flat kernel (1024 words a workgroup, per-lane divmod + index
// load; 4.38 TB/s at n = 32768) this is 5.9 TB/s; 1 or 4 words a thread,
// more words per thread and plain stores were all slower.
// blockIdx.y = 0: state from idx, 1: next_state from idx+1 (N-1 wraps to 0;
// only the last sorted index can, replay.py:160-166) plus one-hot action,
// reward, non_terminal of idx+1.
constexpr int kGatherWpt = 2;
__global__ __launch_bounds__(256) void gather_nchw_kernel(
    const uint8_t* __restrict__ st, const uint8_t* __restrict__ act,
    const int16_t* __restrict__ rew, const uint8_t* __restrict__ nt, ReplayMeta* meta,
    const int32_t* __restrict__ idx, int n, uint32_t wps, FastDiv cpr, float* __restrict__ s0,
    float* __restrict__ s1, float* __restrict__ action, float* __restrict__ reward,
    float* __restrict__ nonterm) {
  typedef float fv4 __attribute__((ext_vector_type(4)));
  const int z = blockIdx.y;
  const int64_t N = meta->capacity;
  uint32_t b, part;
  cpr.divmod(blockIdx.x, b, part);
  const int64_t i = idx[b];
  const int64_t slot = z ? ((i + 1 == N) ? 0 : i + 1) : i;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(st) + (uint64_t)slot * wps;
  fv4* dst = reinterpret_cast<fv4*>(z ? s1 : s0) + (uint64_t)b * wps;
  uint32_t v[kGatherWpt];
#pragma unroll
  for (int k = 0; k < kGatherWpt; ++k) {
    const uint32_t q = part * (256 * kGatherWpt) + k * 256 + threadIdx.x;
    v[k] = q < wps ? src[q] : 0u;
  }
#pragma unroll
  for (int k = 0; k < kGatherWpt; ++k) {
    const uint32_t q = part * (256 * kGatherWpt) + k * 256 + threadIdx.x;
    if (q < wps) {
      const fv4 f = {(float)(v[k] & 255), (float)((v[k] >> 8) & 255),
                     (float)((v[k] >> 16) & 255), (float)(v[k] >> 24)};
      __builtin_nontemporal_store(f, dst + q);
    }
  }
  if (z == 1) {
    const uint32_t r = blockIdx.x * 256 + threadIdx.x;   // first blocks: per-row scalars
    if ((int)r < n) {
      const int64_t j = idx[r];
      const int64_t nxt = (j + 1 == N) ? 0 : j + 1;
      const int a = act[nxt];
      if (a >= kActions) meta->err = 1;
#pragma unroll
      for (int k = 0; k < 4; ++k) action[(size_t)r * 4 + k] = (k == a) ? 1.f : 0.f;
      reward[r] = (float)rew[nxt];
      nonterm[r] = nt[nxt] ? 1.f : 0.f;
    }
  }
}

hipError_t launch_sample_batch(ReplayMeta* meta, int64_t valid, int n, uint64_t seed,
                               uint64_t ctr, uint32_t* bm, int32_t* blk, int32_t* idx,
                               hipStream_t s) {
  const int64_t nwords = (valid + 31) / 32;
  const int nblk = (int)((nwords + 1023) / 1024);
  CHECK_LAUNCH(hipMemsetAsync(bm, 0, (size_t)nblk * 1024 * 4, s));
  ddq_launch(claim_kernel, dim3((n + 255) / 256), dim3(256), 0, s, meta, n, seed, ctr, bm);
  ddq_launch(bm_count_kernel, dim3(nblk), dim3(256), 0, s, bm, nwords, blk);
  ddq_launch(bm_scan_kernel, dim3(1), dim3(256), 0, s, blk, nblk);
  ddq_launch(bm_emit_kernel, dim3(nblk), dim3(256), 0, s, bm, nwords, blk, idx, n);
  return hipGetLastError();
}

hipError_t launch_gather_nchw(const uint8_t* st, const uint8_t* act, const int16_t* rew,
                              const uint8_t* nt, ReplayMeta* meta, const int32_t* idx, int n,
                              int S, float* s0, float* s1, float* action, float* reward,
                              float* nonterm, hipStream_t s) {
  const uint32_t wps = (uint32_t)(S * S);          // 4-byte words per slot
  const uint32_t per = 256u * kGatherWpt;
  const uint32_t cpr = (wps + per - 1) / per;       // n * cpr < 2^31 (n <= 2^31 / S^2 checked)
  ddq_launch(gather_nchw_kernel, dim3((uint32_t)n * cpr, 2), dim3(256), 0, s, st, act, rew, nt,
             meta, idx, n, wps, FastDiv(cpr), s0, s1, action, reward, nonterm);
  return hipGetLastError();
}

// on-device tiling of a transition pool over the ring (1M-slot C5 fills)
__global__ __launch_bounds__(256) void tile_kernel(uint8_t* __restrict__ dst,
                                                   const uint8_t* __restrict__ src,
                                                   uint64_t pool_bytes, uint64_t total) {
  for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16; i < total;
       i += (uint64_t)gridDim.x * 256 * 16) {
    const uint64_t j = i % pool_bytes;
    *reinterpret_cast<uint4*>(dst + i) = *reinterpret_cast<const uint4*>(src + j);
  }
}

hipError_t launch_tile(uint8_t* dst, const uint8_t* src, uint64_t pool_bytes, uint64_t total,
                       hipStream_t s) {
  ddq_launch(tile_kernel, dim3(4096), dim3(256), 0, s, dst, src, pool_bytes, total);
  return hipGetLastError();
}

// u8 (n,4,S,S) -> f32 NHWC (n,S,S,4)  (acting path, select_action)
__global__ void u8_to_nhwc_kernel(const uint8_t* src, int n, int S, float* dst) {
  const int SS = S * S;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * SS) return;
  const int b = i / SS, p = i % SS;
  const uint8_t* s = src + (size_t)b * 4 * SS + p;
  reinterpret_cast<float4*>(dst)[i] = f4(s[0], s[SS], s[2 * SS], s[3 * SS]);
}

hipError_t launch_u8_to_nhwc(const uint8_t* src, int n, int S, float* dst, hipStream_t s) {
  const int tot = n * S * S;
  ddq_launch(u8_to_nhwc_kernel, dim3((tot + 255) / 256), dim3(256), 0, s, src, n, S, dst);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Caffe (co,ci,ky,kx) -> kernel layout (co,ky,kx,ci) for the three convs
// ---------------------------------------------------------------------------
// (the data gradients' transposed + flipped copies, Wt[ci][T-1 - tap][co], are
// made from the forward layout per step: wkst_tap, by the head launch's or the
// deepq16 tower launch's extra workgroups)
struct ConvDims { int64_t w_off, wks_off; int cout, cin, ks; };

// e: Caffe-order element (co, ci, ky, kx) of the layer's weight (< 2^31);
// returns its offset in the split forward layout (split.h):
// conv1 [co][ky][kx 0..7][ci] (kx 7 stays zero), conv2/3 [co][tap][ci]
__device__ __forceinline__ int wks_local(const ConvDims& d, int e) {
  const int kk = d.ks * d.ks, per = d.cin * kk;
  const int co = e / per, rem = e - co * per;
  const int ci = rem / kk, tap = rem - ci * kk;
  if (d.ks == 7) {
    const int ky = tap / 7, kx = tap - 7 * ky;
    return ((co * 7 + ky) * 8 + kx) * 4 + ci;
  }
  return (co * kk + tap) * d.cin + ci;
}

// conv weight element e (of layer d) now holds v: refresh its split forward
// layout (the split data gradients read it transposed, head kernel)
__device__ __forceinline__ void put_conv_weight(const ConvDims& d, int e, float v, __bf16* wks,
                                                int64_t wks_plane) {
  store_split(wks, wks_plane, d.wks_off + wks_local(d, e), v);
}

__global__ void relayout_kernel(const float* __restrict__ theta, __bf16* __restrict__ wks,
                                int64_t wks_plane, ConvDims d0, ConvDims d1, ConvDims d2) {
  const int l = blockIdx.y;
  const ConvDims d = l == 0 ? d0 : (l == 1 ? d1 : d2);
  const int n = d.cout * d.cin * d.ks * d.ks;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x)
    put_conv_weight(d, e, theta[d.w_off + e], wks, wks_plane);
}

static void conv_dims(const ParamLayout& L, ConvDims* d) {
  const int cout[3] = {32, 64, 64}, cin[3] = {4, 32, 64}, ks[3] = {7, 5, 3};
  for (int i = 0; i < 3; ++i) d[i] = {L.w[i], L.wks_off[i], cout[i], cin[i], ks[i]};
}

hipError_t launch_relayout(const NetBuffers& nb, int z, hipStream_t s) {
  ConvDims d[3];
  conv_dims(nb.L, d);
  ddq_launch(relayout_kernel, dim3(64, 3), dim3(256), 0, s, nb.theta[z], nb.wks[z],
                     nb.L.wks_total, d[0], d[1], d[2]);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// fc4 split-K reduce + bias + ReLU (dropout = identity, TEST phase) fused with
// the Q_out / P_out inner product (train_val.prototxt:195-215, :365-383).
// grid (B, nz), 512 threads: thread n owns h4[z][b][n].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(512) void fc4_reduce_out_kernel(
    const float* __restrict__ part, int splits, int nz, int B, const float* __restrict__ b4q,
    const float* __restrict__ b4p, const float* __restrict__ w5q, const float* __restrict__ b5q,
    const float* __restrict__ w5p, const float* __restrict__ b5p, float* __restrict__ h4q,
    float* __restrict__ h4p, float* __restrict__ outq, float* __restrict__ outp) {
  __shared__ float red[8][4];
  const int b = blockIdx.x, z = blockIdx.y, n = threadIdx.x;
  const float* p = part + ((size_t)z * B + b) * kFc4 + n;
  const size_t stride = (size_t)nz * B * kFc4;
  float acc = 0.f;
  int s = 0;
  for (; s + 4 <= splits; s += 4) {
    const float v0 = p[(s + 0) * stride], v1 = p[(s + 1) * stride];
    const float v2 = p[(s + 2) * stride], v3 = p[(s + 3) * stride];
    acc += v0; acc += v1; acc += v2; acc += v3;
  }
  for (; s < splits; ++s) acc += p[s * stride];
  const float v = acc + (z ? b4p : b4q)[n];
  const float h = v > 0.f ? v : 0.f;
  (z ? h4p : h4q)[(size_t)b * kFc4 + n] = h;
  const float* w5 = z ? w5p : w5q;
  float q[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) q[a] = h * w5[a * kFc4 + n];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int a = 0; a < 4; ++a) q[a] += __shfl_xor(q[a], off);
  const int w = n >> 6;
  if ((n & 63) == 0)
#pragma unroll
    for (int a = 0; a < 4; ++a) red[w][a] = q[a];
  __syncthreads();
  if (n < 4) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][n];
    (z ? outp : outq)[b * 4 + n] = t + (z ? b5p : b5q)[n];
  }
}

// ---------------------------------------------------------------------------
// fc4 split-K reduce + bias + ReLU + Q_out (both towers) fused with the head
// and the Q_out backward (train_val.prototxt:169-483), one workgroup per
// sample b (512 threads = the 512 fc4 units):
//   h4 = ReLU(sum_s part + b4), Q/P = W5 h4 + b5,
//   Q_sa = sum_a Q*act, P_sa = max_a P * nt, target = 0.85 P_sa + r,
//   dQ = act (Q_sa-target)/B, dh4 = (dQ W5) * (h4>0).
// The cross-sample sums (loss, dW5, db5, db4) are finished by the head blocks
// of the wgrad slab reduce (per-sample dQ and squared error kept in dqbuf /
// lpart), so the head costs no launch of its own.
// ---------------------------------------------------------------------------
// Blocks [B, B + 25 + 9) of the head launch: conv2's and conv3's split
// forward weights of Q (wks [co][tap][ci], 64 co) transposed + flipped for
// their data gradients (Wt[ci][T-1 - tap][co]), one tap per block through
// LDS, coalesced both ways.  The head is a latency-bound 32-block launch, so
// these blocks ride for free; every step runs its head after the previous
// apply changed the weights and before its conv data gradients.
constexpr int kWkstSmemB = 3 * 64 * (64 + 2) * 2;   // the larger (CI = 64) tile
template <int CI, int T>
__device__ __forceinline__ void wkst_tap(const __bf16* __restrict__ wks, int64_t plane,
                                         int64_t src_off, int64_t dst_off, int t, char* smem) {
  uint16_t (*tile)[64][CI + 2] = reinterpret_cast<uint16_t (*)[64][CI + 2]>(smem);
  constexpr int E = 64 * CI;
  const uint16_t* src = reinterpret_cast<const uint16_t*>(wks) + src_off;
  uint16_t* dst = reinterpret_cast<uint16_t*>(const_cast<__bf16*>(wks)) + dst_off;
  for (int e = threadIdx.x; e < 3 * E; e += blockDim.x) {
    const int p = e / E, r = e % E, co = r / CI, ci = r % CI;
    tile[p][co][ci] = src[p * plane + (co * T + t) * CI + ci];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 3 * E; e += blockDim.x) {
    const int p = e / E, r = e % E, ci = r >> 6, co = r & 63;
    dst[p * plane + (ci * T + T - 1 - t) * 64 + co] = tile[p][co][ci];
  }
}

struct HeadArgs {
  const float* part;
  int splits, B;
  float gamma;
  const float *thq, *thp;
  int64_t b4_off, w5_off, b5_off;
  const float *action, *reward, *nonterm;
  float *h4q, *h4p, *outq, *outp, *q_sa_o, *p_sa_o, *target_o, *dqbuf, *lpart, *dh4;
  int32_t* latch;
  const int64_t* iter;
  int period, inc;
  ReplayMeta* bump;
  const __bf16* wks;
  int64_t wks_plane, wks2_off, wkst_off, wks3_off, wkst3_off;
  // pipelined fused steps: one extra block draws the NEXT step's sorted index
  // set into didx and advances the draw counter (instead of every prefetch
  // block of the slab-reduce launch drawing it again, and block 0 bumping)
  ReplayMeta* dmeta;
  int32_t* didx;
  uint64_t dseed;
  int32_t* dlog;
  int64_t dlog_cap;
};

__device__ __forceinline__ void head_draw(const HeadArgs& H) {
  __shared__ int64_t cand[256];
  __shared__ int bad_any;
  const uint64_t ctr = H.dmeta->counter + 1;     // the advance this launch makes, below
  draw_sorted(H.dmeta, H.B, H.dseed, ctr, cand, &bad_any);
  const int t = threadIdx.x;
  if (t < H.B) {
    H.didx[t] = (int32_t)cand[t];
    log_draw(H.dlog, H.dlog_cap, ctr, H.B, t, (int32_t)cand[t]);
  }
  __syncthreads();                                // every thread has read the counter
  if (t == 0) H.dmeta->counter = ctr;
}

// K1's extra workgroup (small.h): the fused apply's latch, then the draw
// counter's advance or the next step's draw (launch_head's, for S = 16)
namespace sm16 {
__device__ void book_block(const BookArgs& k) {
  if (k.latch && threadIdx.x == 0) {
    k.latch[2] = (k.latch[0] == 0);
    k.latch[3] = k.period > 0 && ((*k.iter + k.inc) % k.period) == 0;
  }
  if (k.dmeta) {
    __shared__ int64_t cand[256];
    __shared__ int bad_any;
    const uint64_t ctr = k.dmeta->counter + 1;
    draw_sorted(k.dmeta, k.B, k.dseed, ctr, cand, &bad_any);
    const int t = threadIdx.x;
    if (t < k.B) {
      k.didx[t] = (int32_t)cand[t];
      log_draw(k.dlog, k.dlog_cap, ctr, k.B, t, (int32_t)cand[t]);
    }
    __syncthreads();
    if (t == 0) k.dmeta->counter = ctr;
  } else if (k.bump && threadIdx.x == 0) {
    k.bump->counter += 1;
  }
}

__device__ void tower_transpose(const TowerArgs& a, int x, char* smem) {
  if (x < 25) wkst_tap<32, 25>(a.wks[0], a.wks_plane, a.wks2_off, a.wkst_off, x, smem);
  else wkst_tap<64, 9>(a.wks[0], a.wks_plane, a.wks3_off, a.wkst3_off, x - 25, smem);
}

hipError_t launch_tower_fwd16(const TowerArgs& t, hipStream_t s) {
  const bool book = t.bk.latch || t.bk.bump || t.bk.dmeta;
  const int extra = (book ? 1 : 0) + t.ntr;
  if (t.xchg && 2 * t.B * t.nz <= 256) {
    // split form: two workgroups per (image, tower), every pair resident at
    // once (<= 256 workgroups of one per CU: their meet cannot wait on an
    // undispatched partner)
    constexpr int K2 = 5, K3 = 4;   // (tap pairs in flight)
    auto kern = tower_fwd16s_kernel<K2, K3>;
    static std::atomic<uint64_t> attr{0};
    if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, kFwdSmemS)) return e;
    ddq_launch(kern, dim3(2 * t.B * t.nz + extra), dim3(kThreads), kFwdSmemS, s, t);
    return hipGetLastError();
  }
  constexpr int K2 = 6, K3 = 5;
  auto kern = tower_fwd16_kernel<K2, K3>;
  static std::atomic<uint64_t> attr{0};
  if (hipError_t e = ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, kFwdSmem)) return e;
  ddq_launch(kern, dim3(t.B * t.nz + extra), dim3(kThreads), kFwdSmem, s, t);
  return hipGetLastError();
}
}  // namespace sm16

// One head block b
__device__ __forceinline__ void head_body(const HeadArgs& H, int b, char* smem) {
  const float* __restrict__ part = H.part;
  const int splits = H.splits, B = H.B;
  const float gamma = H.gamma;
  const float* __restrict__ thq = H.thq;
  const float* __restrict__ thp = H.thp;
  const int64_t b4_off = H.b4_off, w5_off = H.w5_off, b5_off = H.b5_off;
  const float* __restrict__ action = H.action;
  const float* __restrict__ reward = H.reward;
  const float* __restrict__ nonterm = H.nonterm;
  float* __restrict__ h4q = H.h4q;
  float* __restrict__ h4p = H.h4p;
  float* __restrict__ outq = H.outq;
  float* __restrict__ outp = H.outp;
  float *q_sa_o = H.q_sa_o, *p_sa_o = H.p_sa_o, *target_o = H.target_o;
  float* __restrict__ dqbuf = H.dqbuf;
  float* __restrict__ lpart = H.lpart;
  float* __restrict__ dh4 = H.dh4;
  int32_t* latch = H.latch;
  const int64_t* iter = H.iter;
  const int period = H.period, inc = H.inc;
  ReplayMeta* bump = H.bump;
  __shared__ float red[8][8];
  __shared__ float qp[8];
  const int n = threadIdx.x, w = n >> 6;
  if (b == B + 34) {                              // (launched only with dmeta)
    head_draw(H);
    return;
  }
  if (b >= B + 25) {
    wkst_tap<64, 9>(H.wks, H.wks_plane, H.wks3_off, H.wkst3_off, b - B - 25, smem);
    return;
  }
  if (b >= B) {
    wkst_tap<32, 25>(H.wks, H.wks_plane, H.wks2_off, H.wkst_off, b - B, smem);
    return;
  }
  // fused apply: latch the step's apply flags now (the values apply_book
  // latches again in the slab reduce), so the fc4 apply blocks of that launch
  // never read them while its block 0 advances the counters
  if (latch && b == 0 && n == 0) {
    latch[2] = (latch[0] == 0);
    latch[3] = period > 0 && ((*iter + inc) % period) == 0;
  }
  // the step's draw-counter advance (apply_book's bump, moved here): fused
  // apply steps, and async gradients (no apply on the worker)
  if (bump && b == 0 && n == 0) bump->counter += 1;
  const size_t stride = (size_t)2 * B * kFc4;
  float h[2];
  float q[8];
  // every operand that does not depend on the partial sums is loaded first,
  // and the partials 32 splits x 2 towers per round (one round at 64x64):
  // the kernel is a chain of memory latencies, not of work (a quarter of the
  // partials -- 4-wave k-split fc4 forward workgroups -- measured the same
  // 6.4 us here and 6.5 against 6.1 us for the forward)
  float bias4[2], w5v[2][4];
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    const float* th = z ? thp : thq;
    bias4[z] = th[b4_off + n];
#pragma unroll
    for (int a = 0; a < 4; ++a) w5v[z][a] = th[w5_off + a * kFc4 + n];
  }
  float acv[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) acv[a] = action[b * 4 + a];
  const float ntb = nonterm[b], rwb = reward[b];
  // split-K partial sums of both towers, summed in split order
  float acc2[2] = {0.f, 0.f};
  {
    const float* p0 = part + (size_t)b * kFc4 + n;
    const float* p1 = part + ((size_t)B + b) * kFc4 + n;
    for (int s = 0; s < splits; s += 32) {
      float v[2][32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {           // clamped, unconditional loads
        const int su = min(s + u, splits - 1);
        v[0][u] = p0[su * stride];
        v[1][u] = p1[su * stride];
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const bool in = s + u < splits;
        acc2[0] += in ? v[0][u] : 0.f;
        acc2[1] += in ? v[1][u] : 0.f;
      }
    }
  }
#pragma unroll
  for (int z = 0; z < 2; ++z) {
    const float v = acc2[z] + bias4[z];
    h[z] = v > 0.f ? v : 0.f;
    (z ? h4p : h4q)[(size_t)b * kFc4 + n] = h[z];
#pragma unroll
    for (int a = 0; a < 4; ++a) q[z * 4 + a] = h[z] * w5v[z][a];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] += __shfl_xor(q[i], off);
  if ((n & 63) == 0)
#pragma unroll
    for (int i = 0; i < 8; ++i) red[w][i] = q[i];
  __syncthreads();
  if (n < 8) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][n];
    const float* th = n < 4 ? thq : thp;
    t += th[b5_off + (n & 3)];
    qp[n] = t;
    (n < 4 ? outq : outp)[b * 4 + (n & 3)] = t;
  }
  __syncthreads();
  const float* ac = acv;
  // ELTWISE PROD, SLICE, SUM in slice order (train_val.prototxt:386-422)
  float qs = qp[0] * ac[0];
  qs += qp[1] * ac[1];
  qs += qp[2] * ac[2];
  qs += qp[3] * ac[3];
  float ps = fmaxf(fmaxf(qp[4], qp[5]), fmaxf(qp[6], qp[7]));   // SLICE + MAX
  ps = ps * ntb;                                                 // P_sa_or_term
  const float tg = gamma * ps + 1.0f * rwb;                      // SUM coeff {0.85, 1}
  const float diff = qs - tg;
  const float gsc = diff / (float)B;                             // EUCLIDEAN_LOSS diff
  float dq[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) dq[a] = ac[a] * gsc;
  if (n == 0) {
    q_sa_o[b] = qs; p_sa_o[b] = ps; target_o[b] = tg;
    lpart[b] = diff * diff;
#pragma unroll
    for (int a = 0; a < 4; ++a) dqbuf[b * 4 + a] = dq[a];
  }
  const float v = dq[0] * w5v[0][0] + dq[1] * w5v[0][1] + dq[2] * w5v[0][2] + dq[3] * w5v[0][3];
  const float dv = h[0] > 0.f ? v : 0.f;                         // ReLU backward
  dh4[(size_t)b * kFc4 + n] = dv;
}

__global__ __launch_bounds__(512) void fc4_head_kernel(const HeadArgs H) {
  __shared__ __attribute__((aligned(16))) char smem[kWkstSmemB];
  head_body(H, blockIdx.x, smem);
}

// Cross-sample head sums, run by the 8 trailing blocks of the wgrad slab
// reduce: block hb owns fc4 units j = 64 hb + lane, 4 sample groups.
// ---------------------------------------------------------------------------
// apply: server.py update rules on the flat Q tower, float4 per thread, with
//  - the conv kernel-layout copy refreshed from the new values,
//  - the target sync P <- Q fused in when the NEXT pull will see
//    iteration % period == 0 (server.py:188-189),
// ---------------------------------------------------------------------------
struct ApplyArgs {
  int64_t n;
  int64_t lo, hi, skip_lo, skip_len;   // elements [lo, hi) minus [skip_lo, skip_lo + skip_len)
  int rule, period;
  float lr, decay, one_minus_decay, eps, momentum, wd;
  int64_t bias_lo[5], bias_hi[5];   // [lo,hi) element ranges of biases (momentum multipliers)
  ConvDims conv[3];
};

__device__ __forceinline__ float apply_rule(const ApplyArgs& a, bool first, bool is_bias,
                                            float th, float g, float& st);

__device__ __forceinline__ float apply_one(const ApplyArgs& a, bool first, int64_t i, float th,
                                           float g, float& st) {
  bool is_bias = false;
  if (a.rule == 3) {
#pragma unroll
    for (int l = 0; l < 5; ++l) is_bias |= (i >= a.bias_lo[l] && i < a.bias_hi[l]);
  }
  return apply_rule(a, first, is_bias, th, g, st);
}

// the rules themselves; is_bias only matters to the momentum rule
__device__ __forceinline__ float apply_rule(const ApplyArgs& a, bool first, bool is_bias,
                                            float th, float g, float& st) {
  // no FMA contraction: every call site (the apply launch, the fused fc4
  // apply, the shard apply) rounds the rules identically
#pragma clang fp contract(off)
  switch (a.rule) {
    case 0:   // sgd: theta - lr*g  (server.py:81-83, apply_descent :66-68)
      return th - a.lr * g;
    case 1: { // rmsprop with the one-step-lagged cache (server.py:86-105)
      const float g2 = g * g;
      const float c_use = first ? g2 : st;
      st = first ? g2 : (a.decay * st + a.one_minus_decay * g2);
      return th - (a.lr * g) / sqrtf(c_use + a.eps);
    }
    case 2: { // adagrad with the current accumulator (server.py:108-124)
      const float acc = first ? g * g : st + g * g;
      st = acc;
      return th - (a.lr * g) / sqrtf(acc + a.eps);
    }
    default: { // Caffe SGDSolver momentum (blobs_lr {1,2}, weight_decay {1,0})
      const float lr = a.lr * (is_bias ? 2.f : 1.f);
      const float wd = is_bias ? 0.f : a.wd;
      const float v = a.momentum * (first ? 0.f : st) + lr * (g + wd * th);
      st = v;
      return th - v;
    }
  }
}

// Update operands of the apply (the apply launch, or the fused fc4-weight
// apply blocks of the slab-reduce launch).
struct ApplyTail {
  float* theta;
  const float* grad;
  float* opt;
  const int32_t* opt_init;   // [2] first call, [3] P<-Q sync due: latched before the launch
  float* thetaP;
  __bf16* wks;               // split forward weights of Q / P (plane stride wks_plane)
  __bf16* wksP;
  int64_t wks_plane;
  int nfa;                   // slab reduce: fc4 apply blocks (the first of the launch)
  int rest;                  // slab reduce: also update conv / fc4-bias / fc5 params
  int ext;                   // slab reduce: fc4's weight gradient is in grad already
                             // (computed by fc4_bwd, summed over the ranks under the
                             // conv backward): apply from it instead of computing it
  int store_grad;            // fused apply: also store fc4's computed weight gradient
  int64_t w5_off, b5_off, b4_off;
};

__device__ __forceinline__ void apply_at(const ApplyTail& t, const ApplyArgs& a, bool first,
                                         bool sync, int64_t i, float g, float th, float st,
                                         bool is_bias, bool conv = false,
                                         const ConvDims& cd = ConvDims{}, int e = 0);
__device__ __forceinline__ void head_sums(int hb, int B, const float* __restrict__ dqbuf,
                          const float* __restrict__ lpart, const float* __restrict__ h4q,
                          const float* __restrict__ dh4, float* loss_o, float* __restrict__ gw5,
                          float* __restrict__ gb5, float* __restrict__ gb4,
                          bool ap, const ApplyTail& at, const ApplyArgs& aa) {
  __shared__ float red[4 * 64 * 5];
  const int t = threadIdx.x, lane = t & 63, g = t >> 6;
  // fused steps: these sums are final here, so their elements are updated
  // here too (theta / state loaded first, under the sums' loads)
  const int64_t w5_off = at.w5_off, b5_off = at.b5_off, b4_off = at.b4_off;
  const bool first = ap && at.opt_init[2] != 0, sync = ap && at.opt_init[3] != 0;
  float th5[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, st5[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float thb5 = 0.f, stb5 = 0.f;
  if (ap && g == 0) {
    const int jj = hb * 64 + lane;
    th5[0] = at.theta[b4_off + jj];
    if (aa.rule != 0 && !first) st5[0] = at.opt[b4_off + jj];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      th5[1 + a] = at.theta[w5_off + a * kFc4 + jj];
      if (aa.rule != 0 && !first) st5[1 + a] = at.opt[w5_off + a * kFc4 + jj];
    }
  }
  if (ap && hb == 0 && t < 4) {
    thb5 = at.theta[b5_off + t];
    if (aa.rule != 0 && !first) stb5 = at.opt[b5_off + t];
  }
  if (hb == 0 && t < 5) {
    // sequential sums over b, loads issued 16 at a time (clamped indices,
    // dropped): the plain loop was a chain of dependent loads that made
    // these five threads the reduce kernel's critical path (~9 us)
    const float* src = t < 4 ? dqbuf + t : lpart;
    const int es = t < 4 ? 4 : 1;
    float acc = 0.f;
    for (int b0 = 0; b0 < B; b0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = src[min(b0 + u, B - 1) * es];
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (b0 + u < B) acc += v[u];
    }
    if (t < 4) {
      gb5[t] = acc;
      if (ap) apply_at(at, aa, first, sync, b5_off + t, acc, thb5, stb5, true);
    } else {
      *loss_o = acc / (float)B / 2.f;
    }
  }
  const int j = hb * 64 + lane;
  float db = 0.f, dw[4] = {0.f, 0.f, 0.f, 0.f};
  // rounds of 8 batch rows with every load issued first (clamped indices,
  // dropped in the sums); the sums run in the same order as a plain loop
  for (int b0 = g; b0 < B; b0 += 32) {
    float hv[8], dv[8];
    float4 dq[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int bb = min(b0 + 4 * u, B - 1);
      hv[u] = h4q[(size_t)bb * kFc4 + j];
      dv[u] = dh4[(size_t)bb * kFc4 + j];
      dq[u] = *reinterpret_cast<const float4*>(dqbuf + bb * 4);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (b0 + 4 * u >= B) break;
      db += dv[u];
      dw[0] += dq[u].x * hv[u];
      dw[1] += dq[u].y * hv[u];
      dw[2] += dq[u].z * hv[u];
      dw[3] += dq[u].w * hv[u];
    }
  }
  float* r = red + (g * 64 + lane) * 5;
  r[0] = db;
#pragma unroll
  for (int a = 0; a < 4; ++a) r[1 + a] = dw[a];
  __syncthreads();
  if (g == 0) {
    float s[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) s[q] = red[lane * 5 + q];
#pragma unroll
    for (int gg = 1; gg < 4; ++gg)
#pragma unroll
      for (int q = 0; q < 5; ++q) s[q] += red[(gg * 64 + lane) * 5 + q];
    gb4[j] = s[0];
#pragma unroll
    for (int a = 0; a < 4; ++a) gw5[a * kFc4 + j] = s[1 + a];
    if (ap) {
      apply_at(at, aa, first, sync, b4_off + j, s[0], th5[0], st5[0], true);
#pragma unroll
      for (int a = 0; a < 4; ++a)
        apply_at(at, aa, first, sync, w5_off + a * kFc4 + j, s[1 + a], th5[1 + a], st5[1 + a],
                 false);
    }
  }
}

static HeadArgs head_args(const NetBuffers& nb, ReplayMeta* bump) {
  const ParamLayout& L = nb.L;
  return HeadArgs{nb.fc4_part, nb.fc4_splits, nb.B, nb.gamma, nb.theta[0], nb.theta[1], L.b[3],
                  L.w[4], L.b[4], nb.action, nb.reward, nb.nonterm, nb.h4[0], nb.h4[1], nb.q_out,
                  nb.p_out, nb.q_sa, nb.p_sa, nb.target, nb.dqbuf, nb.lpart, nb.dh4,
                  nb.fa.on ? nb.opt_init : nullptr, nb.iter, nb.fa.period, nb.book_inc,
                  (nb.fa.on || nb.head_bump) ? bump : nullptr, nb.wks[0], L.wks_total,
                  L.wks_off[1], L.wkst_off,
                  L.wks_off[2], L.wkst3_off};
}

static Fc4DgradArgs fc4_dgrad_args(const NetBuffers& nb, bool& narrow, int& ndx, int& nd) {
  const int s4 = nb.S / 8, B = nb.B;
  Fc4DgradArgs f;
  f.B = B; f.K = 64 * s4 * s4; f.s4 = s4; f.fS4sq = FastDiv(s4 * s4); f.fS4 = FastDiv(s4);
  f.dh4 = nb.dh4; f.w4 = nb.theta[0] + nb.L.w[3]; f.mask3 = nb.mask3; f.dconv3 = nb.dconv3;
  f.pooled = 1;
  f.dsplit = nullptr;   // conv3's gradients split the fp32 dpool3 themselves
  // 16-column blocks when 32-column ones would not give every CU one
  narrow = (f.K / 32) * ((B + 31) / 32) < 256;
  ndx = f.K / (narrow ? 16 : 32);
  nd = ndx * ((B + 31) / 32);
  return f;
}

hipError_t launch_head(const NetBuffers& nb, hipStream_t s, ReplayMeta* bump, const Prefetch* pf) {
  HeadArgs H = head_args(nb, bump);
  int extra = 0;
  if (pf && pf->ng > 0 && H.bump && nb.B <= 256) {   // the next step's draw moves here
    H.dmeta = H.bump;
    H.bump = nullptr;
    H.didx = pf->idx; H.dseed = pf->seed; H.dlog = pf->idx_log; H.dlog_cap = pf->log_cap;
    extra = 1;
  }
  ddq_launch(fc4_head_kernel, dim3(nb.B + 25 + 9 + extra), dim3(kFc4), 0, s, H);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// conv wgrad slab reduce -> Caffe (co,ci,ky,kx) weight diff + bias diff.
// One workgroup = 64 consecutive slab columns n of one (layer, co) x 4 split
// groups; coalesced slab reads, fixed-order (deterministic) sums, scattered
// writes into the Caffe layout.
// ---------------------------------------------------------------------------
struct WredDims {
  int64_t w_off, b_off, part_off;
  int cout, cin, ks, splits, np, blk0;   // blk0: first workgroup of this layer
  int64_t wks_off;                       // the layer's split layout (fused apply)
  int G;                                 // waves per unit (1, 2 or 4)
};

struct HeadSums {
  int blk0, B;
  const float *dqbuf, *lpart, *h4q, *dh4;
  float *loss, *gw5, *gb5, *gb4;
};

// inc: gradients the apply consumes (param-server iterations: 1, or W in
// the ordered server exchange, server.py:200 INCR per received gradient)
__device__ __forceinline__ void apply_book(int64_t* iter, int32_t* opt_init, int period,
                                           ReplayMeta* bump = nullptr, int inc = 1) {
  if (bump) bump->counter += 1;     // the step's fused draw (sample_gather_kernel)
  const int64_t it = *iter;
  opt_init[2] = (opt_init[0] == 0);
  opt_init[3] = period > 0 && ((it + inc) % period) == 0;
  *iter = it + inc;
  opt_init[0] = 1;
}

// One float4 of parameters per thread: block blk covers elements
// lo + blk*1024 ..., with the skipped range jumped over (float4-aligned).
__device__ __forceinline__ void apply_elems(const ApplyTail& t, const ApplyArgs& a, int64_t blk) {
  const bool first = t.opt_init[2] != 0;
  const bool sync = t.opt_init[3] != 0;
  int64_t i = a.lo + (blk * 256 + threadIdx.x) * 4;
  if (i >= a.skip_lo) i += a.skip_len;
  if (i >= a.hi) return;
  const float4 g4 = *reinterpret_cast<const float4*>(t.grad + i);
  const float4 t4 = *reinterpret_cast<const float4*>(t.theta + i);
  float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.rule != 0 && !first) s4 = *reinterpret_cast<const float4*>(t.opt + i);
  float th[4] = {t4.x, t4.y, t4.z, t4.w};
  const float g[4] = {g4.x, g4.y, g4.z, g4.w};
  float st[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) th[e] = apply_one(a, first, i + e, th[e], g[e], st[e]);
  const float4 o4 = make_float4(th[0], th[1], th[2], th[3]);
  // write-through (split.h wt_store4): no dirty theta / state lines for the
  // launch's end to write back
  const uint32_t nb = (uint32_t)(((a.n + 3) & ~3ll) * 4), ib = (uint32_t)(i * 4);
  wt_store4(wt_rsrc(t.theta, nb), ib, o4);
  if (a.rule != 0) wt_store4(wt_rsrc(t.opt, nb), ib, make_float4(st[0], st[1], st[2], st[3]));
  if (sync) wt_store4(wt_rsrc(t.thetaP, nb), ib, o4);
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const ConvDims& d = a.conv[l];
    const int64_t e0 = i - d.w_off;
    if (e0 >= 0 && e0 < (int64_t)d.cout * d.cin * d.ks * d.ks) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        put_conv_weight(d, (int)e0 + e, th[e], t.wks, t.wks_plane);
        if (sync) put_conv_weight(d, (int)e0 + e, th[e], t.wksP, t.wks_plane);
      }
    }
  }
}

// One element's update in the slab reduce (fused steps): theta / optimizer
// state (loaded by the caller), the P copy on a sync step, and -- for a conv
// weight of layer cd -- its kernel / split layouts.  The caller knows whether
// the element is a bias and which layer it is in, so no range tests here
// (they kept ~20 more scalars live across the reduce and spilled them).
__device__ __forceinline__ void apply_at(const ApplyTail& t, const ApplyArgs& a, bool first,
                                         bool sync, int64_t i, float g, float th, float st,
                                         bool is_bias, bool conv, const ConvDims& cd, int e) {
  th = apply_rule(a, first, is_bias, th, g, st);
  t.theta[i] = th;
  if (a.rule != 0) t.opt[i] = st;
  if (sync) t.thetaP[i] = th;
  if (conv) {
    put_conv_weight(cd, e, th, t.wks, t.wks_plane);
    if (sync) put_conv_weight(cd, e, th, t.wksP, t.wks_plane);
  }
}

// fc4 weight gradient, one (4 R) x 256 tile of dW4[o][k] = sum_n dh4[n][o] x[n][k]
// per 256-thread block: wave w owns rows o0 = 4 R ot + R w .. +R (wave-uniform,
// so dh4 is read through scalar loads), lane owns columns k .. k+3.  Every
// element's sum runs n = 0 .. B-1 in order with fmaf, whatever R, so every
// caller (the gradient launches and the fused apply) produces the same bits.
constexpr int kFc4WTileK = 256;
template <int R>
__host__ __device__ inline int fc4_wgrad_blocks(int K) {
  return (512 / (4 * R)) * ((K + kFc4WTileK - 1) / kFc4WTileK);
}

template <int R>
__device__ __forceinline__ bool fc4_wgrad_coords(int K, int blk, int& o0, int& k) {
  const int nkt = (K + kFc4WTileK - 1) / kFc4WTileK;
  const int ot = blk / nkt, kt = blk - ot * nkt;
  o0 = ot * 4 * R + R * __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  k = kt * kFc4WTileK + 4 * (threadIdx.x & 63);
  return k < K;
}

template <int R>
__device__ __forceinline__ void fc4_wgrad_sum(int B, int K, const float* __restrict__ dh4,
                                              const float* __restrict__ x, int o0, int k,
                                              float (&g)[R][4]) {
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int e = 0; e < 4; ++e) g[r][e] = 0.f;
  const float* xp = x + k;
  const float* dp = dh4 + o0;
#pragma unroll 4   // batch rows per round of loads (8 / 16 measured slower)
  for (int n = 0; n < B; ++n) {
    const float4 xv = *reinterpret_cast<const float4*>(xp + (size_t)n * K);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float d = dp[n * 512 + r];
      g[r][0] = fmaf(d, xv.x, g[r][0]);
      g[r][1] = fmaf(d, xv.y, g[r][1]);
      g[r][2] = fmaf(d, xv.z, g[r][2]);
      g[r][3] = fmaf(d, xv.w, g[r][3]);
    }
  }
}

// Fused fc4-weight apply block (R = 4 rows per wave: 512 blocks at 64x64): the
// tile's theta / optimizer-state loads are issued first so they land under
// the gradient sum; the gradient is written to grad as well (the step's
// gradient stays observable), then the update rule runs (and the P copy on a
// sync step).
constexpr int kFc4ApplyR = 4;   // 2 / 8 rows per wave measured 18.9 / 25.0 us against 13.4
__device__ __forceinline__ void fc4_apply_tile(const ApplyTail& t, const ApplyArgs& a, int B,
                                               int K, const float* dh4, const float* x, int blk) {
  constexpr int R = kFc4ApplyR;
  int o0, k;
  if (!fc4_wgrad_coords<R>(K, blk, o0, k)) return;
  const bool first = t.opt_init[2] != 0;
  const bool sync = t.opt_init[3] != 0;
  const int64_t i0 = a.lo + (int64_t)o0 * K + k;
  // write-through stores (split.h wt_store4): 25 MB per step that would
  // otherwise be written back as dirty L2 lines at the launch's end
  const uint32_t nb = (uint32_t)(a.n * 4);
  const __amdgpu_buffer_rsrc_t rg = wt_rsrc(t.grad, nb), rt = wt_rsrc(t.theta, nb);
  const __amdgpu_buffer_rsrc_t ro = wt_rsrc(t.opt, nb), rp = wt_rsrc(t.thetaP, nb);
  float4 t4[R], s4[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    t4[r] = *reinterpret_cast<const float4*>(t.theta + i0 + (int64_t)r * K);
    s4[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.rule != 0 && !first) s4[r] = *reinterpret_cast<const float4*>(t.opt + i0 + (int64_t)r * K);
  }
  float g[R][4];
  if (t.ext) {   // summed over the ranks already (all-reduce under the conv backward)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float4 g4 = *reinterpret_cast<const float4*>(t.grad + i0 + (int64_t)r * K);
      g[r][0] = g4.x; g[r][1] = g4.y; g[r][2] = g4.z; g[r][3] = g4.w;
    }
  } else {
    fc4_wgrad_sum<R>(B, K, dh4, x, o0, k, g);
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = i0 + (int64_t)r * K;
    const uint32_t ib = (uint32_t)(i * 4);
    if (!t.ext && t.store_grad) wt_store4(rg, ib, make_float4(g[r][0], g[r][1], g[r][2], g[r][3]));
    float th[4] = {t4[r].x, t4[r].y, t4[r].z, t4[r].w};
    float st[4] = {s4[r].x, s4[r].y, s4[r].z, s4[r].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) th[e] = apply_one(a, first, i + e, th[e], g[r][e], st[e]);
    const float4 o4 = make_float4(th[0], th[1], th[2], th[3]);
    wt_store4(rt, ib, o4);
    if (a.rule != 0) wt_store4(ro, ib, make_float4(st[0], st[1], st[2], st[3]));
    if (sync) wt_store4(rp, ib, o4);
  }
}

// Prefetch block g: every block draws the (same) sorted index set of the next
// step with the already-advanced counter, then gathers its slice.
__device__ __forceinline__ void prefetch_body(const Prefetch& pf, int g) {
  __shared__ int64_t cand[256];
  __shared__ int bad_any;
  const int bx = g % pf.gx, b = (g / pf.gx) % pf.B, z = g / (pf.gx * pf.B);
  if (pf.predrawn) {   // the head launch drew the set (head_draw): gather only
    gather_body(pf.st, pf.act, pf.rew, pf.nt, pf.meta, (int64_t)pf.idx[b], pf.S, pf.sQ, pf.sP,
                pf.action, pf.reward, pf.nonterm, bx, b, z);
    return;
  }
  const uint64_t ctr = pf.meta->counter;
  draw_sorted(pf.meta, pf.B, pf.seed, ctr, cand, &bad_any);
  if (g == 0 && threadIdx.x < pf.B) {
    pf.idx[threadIdx.x] = (int32_t)cand[threadIdx.x];
    log_draw(pf.idx_log, pf.log_cap, ctr, pf.B, threadIdx.x, (int32_t)cand[threadIdx.x]);
  }
  gather_body(pf.st, pf.act, pf.rew, pf.nt, pf.meta, cand[b], pf.S, pf.sQ, pf.sP, pf.action,
              pf.reward, pf.nonterm, bx, b, z);
}

// Slab reduce: a unit = 64 slab columns n of one (layer, co), summed over the
// layer's slabs s in the order of four interleaved plain loops (group
// g = s % 4 sums s = g, g+4, ... in turn) combined as (g0 + g1) + (g2 + g3).
// G waves of a block share one unit (G = 1, 2 or 4 per layer, from its slab
// count): wave h of the unit loads slabs s = h, h+G, ... -- at most kWredCh
// in flight per lane, one memory round for this net's slab counts -- into
// 4/G group accumulators, the groups meet in LDS when G > 1.  Every wave
// holds one unit, so the launch is one round deep; measured: persistent
// 4-wave blocks walking 4 units each (one LDS meet per unit) took 5 dependent
// rounds and ~19 us, an (almost) empty launch of ~8000 waves ~4.7 us.
constexpr int kWredCh = 64;

__device__ __forceinline__ int64_t wred_index(const WredDims& d, int lu, int col, int& n,
                                              int& kc) {
  const int nblk = d.np / 64;
  const int co = lu / nblk;
  const int kk = d.ks * d.ks;
  n = (lu % nblk) * 64 + col;
  kc = kk * d.cin;
  return n < kc ? d.w_off + ((int64_t)co * d.cin + n % d.cin) * kk + n / d.cin : d.b_off + co;
}

template <int G>
__device__ __forceinline__ void wred_block(const float* __restrict__ part, float* __restrict__ grad,
                                           const WredDims& d, int lb, float (*red)[4][64],
                                           bool rest, const ApplyTail& fat,
                                           const ApplyArgs& faa) {
  constexpr int NA = 4 / G;   // group accumulators per wave
  // w is per wave: readfirstlane keeps the unit arithmetic scalar
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), col = threadIdx.x & 63;
  const int slot = w / G, h = w % G;
  const int lu = lb * NA + slot;
  int n, kc;
  const int64_t idx = wred_index(d, lu, col, n, kc);
  const bool live = n <= kc;   // slab padding columns (n > kc) are never read
  // fused steps: the unit's element is updated here once its gradient is
  // final; theta / state are loaded before the slab loads
  const bool first = rest && fat.opt_init[2] != 0, sync = rest && fat.opt_init[3] != 0;
  float th = 0.f, st = 0.f;
  if (rest && h == 0 && live) {
    th = fat.theta[idx];
    if (faa.rule != 0 && !first) st = fat.opt[idx];
  }
  float acc[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) acc[j] = 0.f;
  if (live) {
    const int co = lu / (d.np / 64);
    const float* p = part + d.part_off + (size_t)co * d.np + n;
    const size_t stride = (size_t)d.cout * d.np;
    const int cnt = (d.splits - h + G - 1) / G;          // this wave's slabs h + G i
    for (int i0 = 0; i0 < cnt; i0 += kWredCh) {
      float v[kWredCh];
#pragma unroll
      for (int u = 0; u < kWredCh; ++u)                 // clamped, unconditional
        v[u] = p[(size_t)(h + G * min(i0 + u, cnt - 1)) * stride];
#pragma unroll
      for (int u = 0; u < kWredCh; ++u)                 // slab h + G (i0 + u): group
        if (i0 + u < cnt) acc[u % NA] += v[u];          // h + G (u % NA)
    }
  }
  float v;
  if constexpr (G == 1) {
    v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  } else {
#pragma unroll
    for (int j = 0; j < NA; ++j) red[slot][h + G * j][col] = acc[j];
    __syncthreads();
    v = (red[slot][0][col] + red[slot][1][col]) + (red[slot][2][col] + red[slot][3][col]);
  }
  if (h == 0 && live) {
    grad[idx] = v;
    if (rest) {
      const ConvDims cd{d.w_off, d.wks_off, d.cout, d.cin, d.ks};
      const bool wt = n < kc;
      apply_at(fat, faa, first, sync, idx, v, th, st, !wt, wt, cd, (int)(idx - d.w_off));
    }
  }
}

// Reduce blocks [d.blk0, ...) of each layer (conv1, conv3, conv2 order: d0 <
// d2 < d1; a block holds 4 / G units), blocks [nub, nub + 8) the head sums;
// block 0 also latches the apply bookkeeping.  Fused steps (fat.rest) update
// every parameter here, where its gradient becomes final -- no separate apply
// launch.
__global__ __launch_bounds__(256, 4) void wgrad_reduce_kernel(
    const float* __restrict__ part, float* __restrict__ grad, WredDims d0, WredDims d1,
    WredDims d2, int nub, int64_t* iter, int32_t* opt_init, int book_period,
    ReplayMeta* bump, int book_inc, HeadSums hs, ApplyTail fat, ApplyArgs faa, Prefetch pf,
    const float* __restrict__ fc4_x, int fc4_k) {
  __shared__ float red[4][4][64];
  int bid = blockIdx.x;
  // block order: the next step's draw + gather (fused apply), then the head
  // sums' dependent latency chains (behind 800+ HBM-streaming blocks they
  // cost 3 us: reduce 19.4 -> 16.4), then the fused fc4-weight apply tiles
  // (the longest HBM streams start before the slab units: the other order
  // measured 16.6 -> 22.6 us), then the slab units
  if (bid < pf.ng) {
    prefetch_body(pf, bid);
    return;
  }
  bid -= pf.ng;
  const bool rest = fat.rest != 0;
  if (bid < kFc4 / 64) {
    if (opt_init && bid == 0 && threadIdx.x == 0)
      apply_book(iter, opt_init, book_period, bump, book_inc);
    head_sums(bid, hs.B, hs.dqbuf, hs.lpart, hs.h4q, hs.dh4, hs.loss, hs.gw5, hs.gb5, hs.gb4,
              rest, fat, faa);
    return;
  }
  bid -= kFc4 / 64;
  if (bid < fat.nfa) {
    fc4_apply_tile(fat, faa, hs.B, fc4_k, hs.dh4, fc4_x, bid);
    return;
  }
  bid -= fat.nfa;
  // (by value: a reference to a runtime-chosen kernel argument put the
  // three in scratch memory)
  const WredDims d = bid >= d1.blk0 ? d1 : (bid >= d2.blk0 ? d2 : d0);
  if (d.G == 1)
    wred_block<1>(part, grad, d, bid - d.blk0, red, rest, fat, faa);
  else if (d.G == 2)
    wred_block<2>(part, grad, d, bid - d.blk0, red, rest, fat, faa);
  else
    wred_block<4>(part, grad, d, bid - d.blk0, red, rest, fat, faa);
}

// Blocks [0, pf.ng) of the apply launch draw + gather the NEXT step's
// minibatch into the other buffer set (pipelined stepping, B <= 256): the
// sample_gather kernel's work rides on the HBM-bound apply instead of being a
// serial latency-bound launch at the head of the next step.  The counter it
// draws with was advanced by this step's bookkeeping (the reduce kernel), so
// the draws are the ones sequential steps make.
__global__ __launch_bounds__(256) void apply_kernel(ApplyTail t, ApplyArgs a, Prefetch pf) {
  if ((int)blockIdx.x < pf.ng) {
    prefetch_body(pf, blockIdx.x);
    return;
  }
  // (two float4 per thread with every load first measured 12.0 us against 11.3)
  apply_elems(t, a, (int)blockIdx.x - pf.ng);
}

// param-server iteration / first-call bookkeeping of one apply: latch the
// apply's flags (opt_init[2] = first call, opt_init[3] = P<-Q sync due) from
// the old counters, then advance them.  Runs before the apply, either folded
// into the step's wgrad slab reduce or as this one-thread kernel.
__global__ void apply_book_kernel(int64_t* iter, int32_t* opt_init, int period) {
  apply_book(iter, opt_init, period);
}

// Owner apply of one parameter shard [off, off+len) (sharded / server
// exchanges): the W gradient slices gsl[w][0..len) are applied one after the
// other in rank (ticket) order -- server.py:196-209 applies every received
// gradient on arrival (apply_descent :49-78) -- with theta and the optimizer
// state held in registers across the W updates.  Only the first gradient of
// the first apply takes the rules' first-call branch.  Conv kernel layouts and
// the P tower are refreshed after the all-gather (refresh_kernel).
// first >= 0: the rules' first-call flag given by the host (async owner
// applies, whose bookkeeping is this kernel's: block 0 advances the iteration
// and marks the state initialised -- nothing in the launch reads either)
// Blocks [0, pf.ng): the next step's draw + gather (pipelined sharded /
// server steps: the step's bookkeeping in the slab reduce advanced the draw
// counter already).
// launch_refresh's per-float4 work: the P copy on a sync step and, for conv
// weights, the kernel layouts of Q (and P on a sync step)
__device__ __forceinline__ void refresh_elems(const ApplyArgs& a, bool sync, int64_t i,
                                              const float (&th)[4], float* __restrict__ thetaP,
                                              __bf16* wks, __bf16* wksP, int64_t wks_plane) {
  if (sync)
    wt_store4(wt_rsrc(thetaP, (uint32_t)(((a.n + 3) & ~3ll) * 4)), (uint32_t)(i * 4),
              make_float4(th[0], th[1], th[2], th[3]));
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const ConvDims& d = a.conv[l];
    const int64_t e0 = i - d.w_off;
    if (e0 >= 0 && e0 < (int64_t)d.cout * d.cin * d.ks * d.ks) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        put_conv_weight(d, (int)e0 + e, th[e], wks, wks_plane);
        if (sync) put_conv_weight(d, (int)e0 + e, th[e], wksP, wks_plane);
      }
    }
  }
}

struct RefreshOut {
  float* thetaP;
  __bf16* wks;
  __bf16* wksP;
  int64_t wks_plane;
  int mode;   // 0 off; 1 sync = the latched flag; 2 / 3 sync decided by the host: no / yes
};

__global__ __launch_bounds__(256) void apply_shard_kernel(
    float* __restrict__ theta, const float* __restrict__ gsl, float* __restrict__ opt,
    int32_t* __restrict__ opt_init, int64_t off, int64_t len, int64_t slice, int W,
    ApplyArgs a, int first_host, int64_t* iter, Prefetch pf, float* __restrict__ mirror,
    RefreshOut ro, int own_w, const float* __restrict__ own_g) {
  if ((int)blockIdx.x < pf.ng) {
    prefetch_body(pf, blockIdx.x);
    return;
  }
  const int bid = (int)blockIdx.x - pf.ng;
  const bool first = first_host >= 0 ? first_host != 0 : opt_init[2] != 0;
  if (first_host >= 0 && bid == 0 && threadIdx.x == 0) {
    *iter += 1;
    opt_init[0] = 1;
  }
  const int64_t j = ((int64_t)bid * blockDim.x + threadIdx.x) * 4;
  if (j >= len) return;
  const int64_t i = off + j;
  const float4 t4 = *reinterpret_cast<const float4*>(theta + i);
  float4 s4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.rule != 0 && !first) s4 = *reinterpret_cast<const float4*>(opt + i);
  float th[4] = {t4.x, t4.y, t4.z, t4.w};
  float st[4] = {s4.x, s4.y, s4.z, s4.w};
  for (int w = 0; w < W; ++w) {
    // (slice own_w: read in place from the rank's own gradient, not received)
    const float* gw = w == own_w ? own_g : gsl + (int64_t)w * slice;
    const float4 g4 = *reinterpret_cast<const float4*>(gw + j);
    const float g[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      th[e] = (i + e < a.n) ? apply_one(a, first && w == 0, i + e, th[e], g[e], st[e]) : 0.f;
  }
  const uint32_t nb = (uint32_t)((off + len) * 4), ib = (uint32_t)(i * 4);   // the shard's end
  wt_store4(wt_rsrc(theta, nb), ib, make_float4(th[0], th[1], th[2], th[3]));
  if (a.rule != 0) wt_store4(wt_rsrc(opt, nb), ib, make_float4(st[0], st[1], st[2], st[3]));
  // (async owner applying its own worker's push: the worker's copy of the
  // shard too, instead of a pull copy after the apply)
  if (mirror) wt_store4(wt_rsrc(mirror, nb), ib, make_float4(th[0], th[1], th[2], th[3]));
  if (ro.mode)
    refresh_elems(a, ro.mode == 1 ? opt_init[3] != 0 : ro.mode == 3, i, th, ro.thetaP, ro.wks,
                  ro.wksP, ro.wks_plane);
}

// After the theta all-gather: conv kernel layouts of Q, and P <- Q (weights
// and kernel layouts) when the step's bookkeeping latched a target sync.
// force >= 0: the P <- Q decision given by the host (async exchange pulls)
__global__ __launch_bounds__(256) void refresh_kernel(const float* __restrict__ theta,
                                                      const int32_t* __restrict__ opt_init,
                                                      float* __restrict__ thetaP, __bf16* wks,
                                                      __bf16* wksP, int64_t wks_plane,
                                                      ApplyArgs a, int force, int64_t skip_lo,
                                                      int64_t skip_hi) {
  const bool sync = force >= 0 ? force != 0 : opt_init[3] != 0;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= a.n || (i >= skip_lo && i < skip_hi) ||
      (!sync && i >= a.conv[2].w_off + (int64_t)a.conv[2].cout * a.conv[2].cin * 9))
    return;
  const float4 o4 = *reinterpret_cast<const float4*>(theta + i);
  const float th[4] = {o4.x, o4.y, o4.z, o4.w};
  refresh_elems(a, sync, i, th, thetaP, wks, wksP, wks_plane);
}

// out[0..len) = sum_w in[w][0..len) in rank order (in-process group exchange)
__global__ __launch_bounds__(256) void sum_slices_kernel(float* __restrict__ out,
                                                         const float* __restrict__ in, int W,
                                                         int64_t len, int64_t slice) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= len) return;
  float acc = in[j];
  for (int w = 1; w < W; ++w) acc += in[(int64_t)w * slice + j];
  out[j] = acc;
}

static ApplyArgs apply_args(const NetBuffers& nb, int rule, float lr, float decay, float eps,
                            float momentum, float wd, int period) {
  ApplyArgs a;
  a.n = nb.L.total;
  a.lo = 0; a.hi = a.n; a.skip_lo = a.n; a.skip_len = 0;
  a.rule = rule; a.period = period;
  a.lr = lr; a.decay = decay; a.eps = eps; a.momentum = momentum; a.wd = wd;
  a.one_minus_decay = (float)(1.0 - (double)decay);   // numpy: (1 - rmsprop_decay) in double
  for (int l = 0; l < 5; ++l) { a.bias_lo[l] = nb.L.b[l]; a.bias_hi[l] = nb.L.b[l] + nb.L.bn[l]; }
  conv_dims(nb.L, a.conv);
  return a;
}

static ApplyTail apply_tail(const NetBuffers& nb) {
  ApplyTail t{};
  t.theta = nb.theta[0]; t.grad = nb.grad; t.opt = nb.opt; t.opt_init = nb.opt_init;
  t.thetaP = nb.theta[1]; t.wks = nb.wks[0]; t.wksP = nb.wks[1]; t.wks_plane = nb.L.wks_total;
  t.w5_off = nb.L.w[4]; t.b5_off = nb.L.b[4]; t.b4_off = nb.L.b[3];
  t.store_grad = 1;
  return t;
}

// The fused fc4-weight apply (NetBuffers::fa): fc4's weight gradient is final
// after the fc4 backward, so its update runs as extra blocks of the slab-
// reduce launch and the apply launch keeps the rest of the parameters.
bool fused_apply_ok(const ParamLayout& L) {
  return L.w[3] % 4 == 0 && L.b[3] % 4 == 0 && L.b[3] > L.w[3];
}

hipError_t launch_apply_shard(const NetBuffers& nb, int rule, float lr, float decay, float eps,
                              float momentum, float wd, const float* gsl, int64_t off,
                              int64_t len, int64_t slice, int W, hipStream_t s, float* theta,
                              int first, const Prefetch* pre, float* mirror, int refresh_own,
                              int own_w, const float* own_g) {
  const ApplyArgs a = apply_args(nb, rule, lr, decay, eps, momentum, wd, 0);
  Prefetch pf{};
  if (pre) pf = *pre;
  // (shard starts are multiples of 64: a float4 never straddles two shards)
  const RefreshOut ro{nb.theta[1], nb.wks[0], nb.wks[1], nb.L.wks_total,
                      refresh_own < 0 ? 1 : refresh_own == 0 ? 0 : refresh_own == 1 ? 2 : 3};
  const int64_t blocks = (len / 4 + 255) / 256;
  if (blocks + pf.ng > 0)
    ddq_launch(apply_shard_kernel, dim3((uint32_t)(blocks + pf.ng)), dim3(256), 0, s,
                       theta ? theta : nb.theta[0], gsl, nb.opt, nb.opt_init, off, len, slice, W,
                       a, first, nb.iter, pf, mirror, ro, own_g ? own_w : -1, own_g);
  return hipGetLastError();
}


hipError_t launch_refresh(const NetBuffers& nb, hipStream_t s, int force_sync, int64_t skip_lo,
                          int64_t skip_hi) {
  const ApplyArgs a = apply_args(nb, 0, 0.f, 0.f, 0.f, 0.f, 0.f, 0);
  if (skip_lo <= 0 && skip_hi >= a.n) return hipSuccess;
  ddq_launch(refresh_kernel, dim3((uint32_t)((a.n / 4 + 255) / 256)), dim3(256), 0, s,
                     nb.theta[0], nb.opt_init, nb.theta[1], nb.wks[0], nb.wks[1],
                     nb.L.wks_total, a, force_sync, skip_lo, skip_hi);
  return hipGetLastError();
}

hipError_t launch_book(const NetBuffers& nb, int period, hipStream_t s) {
  ddq_launch(apply_book_kernel, dim3(1), dim3(1), 0, s, nb.iter, nb.opt_init, period);
  return hipGetLastError();
}

hipError_t launch_sum_slices(float* out, const float* in, int W, int64_t len, int64_t slice,
                             hipStream_t s) {
  ddq_launch(sum_slices_kernel, dim3((uint32_t)((len + 255) / 256)), dim3(256), 0, s, out,
                     in, W, len, slice);
  return hipGetLastError();
}

Prefetch make_prefetch(const NetBuffers& next, const uint8_t* st, const uint8_t* act,
                       const int16_t* rew, const uint8_t* nt, ReplayMeta* meta, uint64_t seed) {
  Prefetch pf;
  pf.st = st; pf.act = act; pf.rew = rew; pf.nt = nt; pf.meta = meta; pf.seed = seed;
  pf.B = next.B; pf.S = next.S;
  pf.predrawn = 0;
  pf.gx = (next.S * next.S / 4 + 255) / 256;
  pf.ng = pf.gx * next.B * 2;
  pf.idx = next.idx; pf.sQ = next.state; pf.sP = next.next_state;
  pf.idx_log = next.idx_log; pf.log_cap = next.log_cap;
  pf.action = next.action; pf.reward = next.reward; pf.nonterm = next.nonterm;
  return pf;
}

hipError_t launch_apply(const NetBuffers& nb, int rule, float lr, float decay, float eps,
                        float momentum, float wd, int period, bool booked, hipStream_t s,
                        const Prefetch* pre) {
  Prefetch pf{};
  if (pre) pf = *pre;
  ApplyArgs a = apply_args(nb, rule, lr, decay, eps, momentum, wd, period);
  if (!booked) ddq_launch(apply_book_kernel, dim3(1), dim3(1), 0, s, nb.iter, nb.opt_init, period);
  // fused steps: the slab-reduce launch already updated every parameter --
  // or, with its fc4 gradient summed over the ranks under the conv backward
  // (fa.ext), fc4's weights: the rest (summed after the reduce) here
  if (nb.fa.on && nb.fa.ext) { a.skip_lo = nb.L.w[3]; a.skip_len = nb.L.wn[3]; }
  const int blocks = (nb.fa.on && !nb.fa.ext) ? 0 : (int)(((a.n - a.skip_len) / 4 + 255) / 256);
  if (blocks + pf.ng == 0) return hipSuccess;
  ddq_launch(apply_kernel, dim3(blocks + pf.ng), dim3(256), 0, s, apply_tail(nb), a, pf);
  return hipGetLastError();
}

}  // namespace ddq
#include "small_bwd.h"
namespace ddq {

// ---------------------------------------------------------------------------
// layer geometry
// ---------------------------------------------------------------------------
int fc4_splits_for(int S) { return fc4_fwd_splits(64 * (S / 8) * (S / 8)); }

// Tile menus of the direct convolutions.  A tile's rows (its pixels, padded to
// whole 32-row blocks: split.h SplitCfg::NWIN) are the MFMA work of one
// workgroup; the frame's edge tiles of a fixed 16 x 16 tile wasted up to 2.56x
// of it (conv2 at S = 40: four 16 x 16 tiles on a 20 x 20 map).  Per layer and
// map side the cheapest option is taken: tiles x (rows + 32), the 32 standing
// for a workgroup's fixed costs (weight ring, prologue); the first option (the
// tuned tile of the exact 64 x 64 / 128 x 128 frames) is left only for one at
// least 10 % cheaper.
struct TileOpt {
  int ty, tx, rows;
};
template <int CPT, int CP, int N, int KS, int TY, int TX, int WM, int WN, int WK, int MF = 0>
constexpr TileOpt split_tile() {
  return {TY, TX, WM * SplitCfg<CPT, CP, N, KS, TY, TX, WM, WN, WK, MF>::TM * 32};
}
template <int TY, int TX, int WM>
constexpr TileOpt conv1_tile() { return {TY, TX, WM * Conv1Cfg<TY, TX, WM>::TM * 32}; }

template <class T, int n>
static const T& pick_tile(const T (&menu)[n], int H, int W) {
  auto cost = [&](const TileOpt& o) {
    return (int64_t)((H + o.ty - 1) / o.ty) * ((W + o.tx - 1) / o.tx) * (o.rows + 32);
  };
  const int64_t c0 = cost(menu[0].opt);
  int best = 0;
  int64_t bc = c0;
  for (int i = 1; i < n; ++i) {
    const int64_t c = cost(menu[i].opt);
    if (10 * c < 9 * c0 && c < bc) { bc = c; best = i; }
  }
  return menu[best];
}

struct SplitMenu {
  TileOpt opt;
  hipError_t (*launch)(SplitArgs, int, hipStream_t);
};
#define DDQ_SPLIT_TILE(CPT, CP, N, KS, TY, TX, WM, WN, WK, DG, MF)     \
  SplitMenu {                                                         \
    split_tile<CPT, CP, N, KS, TY, TX, WM, WN, WK, MF>(),             \
        &launch_split_conv<CPT, CP, N, KS, TY, TX, WM, WN, WK, DG, MF> \
  }
// conv2 forward (32 -> 64, 5x5): 16 waves of one 32x32 block on 16 x 16, on
// v_mfma_f32_16x16x32_bf16 (MF 1; split.h SplitCfg): 30.1 -> 26.3 us against
// the 32x32x16 form at 64x64, same-box A/B (the chip holds a higher clock on
// the 16x16 shape, MI355X_MICROARCH.md DVFS item 7)
static const SplitMenu kConv2Fwd[] = {
    DDQ_SPLIT_TILE(32, 32, 64, 5, 16, 16, 8, 2, 1, false, 1),
    DDQ_SPLIT_TILE(32, 32, 64, 5, 10, 20, 7, 2, 1, false, 1),
    DDQ_SPLIT_TILE(32, 32, 64, 5, 12, 12, 5, 2, 1, false, 1),
    // small maps (one tile per image): two k groups halve a workgroup's serial
    // tap chain (32x32x16: 16-channel k-steps split, as 16x16x32's cannot be);
    // deepq16 conv2 forward 12.6 -> 11.0 us, same-box A/B
    DDQ_SPLIT_TILE(32, 32, 64, 5, 8, 8, 2, 2, 2, false, 0),
    DDQ_SPLIT_TILE(32, 32, 64, 5, 8, 26, 7, 2, 1, false, 1),
    DDQ_SPLIT_TILE(32, 32, 64, 5, 14, 14, 7, 2, 1, false, 1)};
// conv3 forward (64 -> 64, 3x3): two k groups on 8 x 8
static const SplitMenu kConv3Fwd[] = {
    DDQ_SPLIT_TILE(64, 64, 64, 3, 8, 8, 2, 2, 2, false, 1),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 10, 10, 4, 2, 2, false, 1),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 12, 12, 5, 2, 1, false, 1),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 6, 18, 4, 2, 2, false, 1),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 4, 4, 1, 2, 2, false, 1),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 6, 26, 5, 2, 1, false, 0)};   // (MF 1 exceeds LDS)
// conv3 data gradient: four k groups on 4 x 8
static const SplitMenu kConv3Dgrad[] = {
    DDQ_SPLIT_TILE(64, 64, 64, 3, 4, 8, 1, 2, 4, true, 0),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 6, 10, 2, 2, 4, true, 0),
    DDQ_SPLIT_TILE(64, 64, 64, 3, 6, 26, 5, 2, 1, true, 0)};
// conv2 data gradient (64 -> 32): four k groups on 8 x 16
static const SplitMenu kConv2Dgrad[] = {
    DDQ_SPLIT_TILE(64, 64, 32, 5, 8, 16, 4, 1, 4, true, 0),
    DDQ_SPLIT_TILE(64, 64, 32, 5, 8, 20, 5, 1, 2, true, 0),
    DDQ_SPLIT_TILE(64, 64, 32, 5, 12, 12, 5, 1, 2, true, 0),
    DDQ_SPLIT_TILE(64, 64, 32, 5, 8, 8, 2, 1, 4, true, 0)};
#undef DDQ_SPLIT_TILE

struct Conv1Menu {
  TileOpt opt;
  hipError_t (*launch)(Conv1Args, int, hipStream_t, int64_t);
};
#define DDQ_CONV1_TILE(TY, TX, WM) \
  Conv1Menu { conv1_tile<TY, TX, WM>(), &launch_split_conv1<TY, TX, WM> }
static const Conv1Menu kConv1Fwd[] = {DDQ_CONV1_TILE(32, 32, 16), DDQ_CONV1_TILE(20, 20, 13),
                                      DDQ_CONV1_TILE(16, 16, 8), DDQ_CONV1_TILE(24, 24, 9)};
#undef DDQ_CONV1_TILE

// Slabs of the conv weight gradients and their pitch np (>= KC + 1: the bias
// column, padded to 64 for the reduce's units).  conv1: one per tile of
// conv2's data gradient (the fused conv1 weight gradient, split.h
// w1_tile_wgrad); conv2 / conv3: one per row group (wgrads_groups).
int wgrad_splits_for(int layer, int B, int S, int* np) {
  const int H = S >> layer;
  const int KC[3] = {196, 800, 576};
  *np = ((KC[layer] + 1 + 63) / 64) * 64;
  if (layer == 0) {
    const TileOpt& t = pick_tile(kConv2Dgrad, S / 2, S / 2).opt;
    return B * ((S / 2 + t.ty - 1) / t.ty) * ((S / 2 + t.tx - 1) / t.tx);
  }
  const int nts[3] = {0, 2 * 5, 2 * 3};
  // about 256 workgroups each (24 / 40 slabs at 64x64 B=32: fewer, larger
  // slabs than at 512 -- pair 30.0 -> 27.7 us, reduce 21.9 -> 19.2)
  int target = 256;
  // 16 x 16 maps: at least 16 rows per group -- a slab is the whole weight
  // matrix whatever the rows behind it (deepq16: conv3 on 8 slabs instead of
  // 40, conv2 on 16 instead of 24; 0.0915 -> 0.0896 ms per step, same-box
  // A/B; at 32 x 32 the same rule measured 0.1238 -> 0.1247)
  if (S <= 16) target = std::min(target, std::max(nts[layer], nts[layer] * (B * H) / 16));
  int G, RPG;
  wgrads_groups(B * H, nts[layer], &G, &RPG, target);
  return G;
}

// fc4 data gradient (blocks [0, nd): fc4_dgrad_body, 512 threads) beside the
// fc4 weight gradient (blocks [nd, ...): 256 threads; the other 4 waves end at
// once, which s_barrier does not wait for).  nd = 0 blocks of the weight
// gradient when the fused apply computes it tile by tile itself.
template <bool SPLIT, int KCW>
__global__ __launch_bounds__(512) void fc4_bwd_kernel(const Fc4DgradArgs d, const float* x,
                                                      float* gw4, int nd, int ndx) {
  __shared__ __attribute__((aligned(16))) float smem[8 * 1024];
  const int bid = blockIdx.x;
  if (bid < nd) {
    int lb = bid;
    if (KCW == 16 && nd % 16 == 0) {
      // 16-column blocks 2m and 2m+1 read the two halves of the same 128-byte
      // W4 lines: dispatch them to one XCD (workgroup i runs on XCD i % 8), so
      // that XCD's L2 fetches each line once
      const int xcd = bid & 7, q = bid >> 3;
      lb = 16 * (q >> 1) + 2 * xcd + (q & 1);
    }
    fc4_dgrad_body<SPLIT, KCW>(d, reinterpret_cast<float(*)[1024]>(smem), lb % ndx, lb / ndx);
    return;
  }
  if (threadIdx.x >= 256) return;
  float g[8][4];
  int o0, k;
  if (!fc4_wgrad_coords<8>(d.K, bid - nd, o0, k)) return;
  fc4_wgrad_sum<8>(d.B, d.K, d.dh4, x, o0, k, g);
#pragma unroll
  for (int r = 0; r < 8; ++r)
    *reinterpret_cast<float4*>(gw4 + (size_t)(o0 + r) * d.K + k) =
        make_float4(g[r][0], g[r][1], g[r][2], g[r][3]);
}

// K1 of the S = 16 step (small.h); bk: its extra workgroup's bookkeeping
static sm16::TowerArgs tower_args(const NetBuffers& nb, int nz, const sm16::BookArgs* bk) {
  const ParamLayout& L = nb.L;
  sm16::TowerArgs t{};
  t.B = nb.B; t.nz = nz;
  t.in[0] = nb.state; t.in[1] = nb.next_state;
  for (int z = 0; z < 2; ++z) {
    t.wks[z] = nb.wks[z];
    t.bias1[z] = nb.theta[z] + L.b[0];
    t.bias2[z] = nb.theta[z] + L.b[1];
    t.bias3[z] = nb.theta[z] + L.b[2];
    t.pool3[z] = nb.pool3[z];
  }
  t.wks_plane = L.wks_total; t.wks_off2 = L.wks_off[1]; t.wks_off3 = L.wks_off[2];
  t.pool1s = nb.pool1s[0]; t.pool2s = nb.pool2s[0];
  t.mask1 = nb.mask1; t.mask2 = nb.mask2; t.mask3 = nb.mask3;
  if (bk) t.bk = *bk;
  t.xchg = nb.xchg; t.pairc = nb.pairc;
  t.timeout = nb.csync ? nb.csync + 48 : nullptr;   // (csync: allocated at S = 16)
  // K3's transposed weights, from this launch's Q weights (its extra blocks)
  t.ntr = 25 + 9;
  t.wks2_off = L.wks_off[1]; t.wkst_off = L.wkst_off;
  t.wks3_off = L.wks_off[2]; t.wkst3_off = L.wkst3_off;
  return t;
}

hipError_t launch_forward(const NetBuffers& nb, int nz, hipStream_t s,
                          void (*mark)(void*, const char*), void* marg, bool out) {
  const ParamLayout& L = nb.L;
  const int B = nb.B, S = nb.S;
  auto M = [&](const char* n) { if (mark) mark(marg, n); };
  const float* in[2] = {nb.state, nb.next_state};
  // deepq16: conv1 -> pool3 of each (image, tower) in one workgroup (small.h)
  const bool tower = !nb.fwd_only && nb.small;
  if (tower) {
    M("tower_fwd");
    CHECK_LAUNCH(sm16::launch_tower_fwd16(tower_args(nb, nz, nullptr), s));
  }
  if (!tower && (!nb.fwd_only || nb.fwd_only == 1)) {
    // conv1 (train_val.prototxt:39-78): bf16 matrix cores, fp32-exact
    // (split.h): frames are exact in bf16, so 3 MFMAs per 32x32x16 block; the
    // pooled output goes out fp32 NHWC (conv2 splits it while staging and
    // writes the Q tower's split for conv2's weight gradient)
    Conv1Args c1{};
    c1.B = B; c1.H = S; c1.W = S;
    for (int z = 0; z < 2; ++z) {
      c1.in[z] = in[z];
      c1.wk[z] = nb.wks[z] + L.wks_off[0];
      c1.bias[z] = nb.theta[z] + L.b[0];
      c1.out[z] = nb.pool1f[z];
    }
    c1.out_split[0] = c1.out_split[1] = nullptr;
    c1.out_elems = (int64_t)B * (S / 2) * (S / 2) * 32;
    c1.mask[0] = nb.mask1; c1.mask[1] = nullptr;
    M("conv1_fwd");
    CHECK_LAUNCH(pick_tile(kConv1Fwd, S, S).launch(c1, nz, s, L.wks_total));
  }
  if (!tower && (!nb.fwd_only || nb.fwd_only == 2)) {
    // conv2 (train_val.prototxt:79-118): split bf16, 16x16 tiles, 16 waves of
    // one 32x32 block each (kConv2Fwd: edge-fitting tiles on other maps)
    const int H = S / 2;
    SplitArgs a2{};
    a2.B = B; a2.H = H; a2.W = H; a2.pad = 2;
    for (int z = 0; z < 2; ++z) {
      a2.in32[z] = nb.pool1f[z];
      a2.wk[z] = nb.wks[z] + L.wks_off[1];
      a2.bias[z] = nb.theta[z] + L.b[1];
      a2.out[z] = nb.pool2f[z];   // fp32 NHWC (conv3 splits it while staging)
    }
    a2.wk_elems = L.wks_total;
    // the Q tower's staged input, split, for conv2's weight gradient
    a2.xsplit = nb.pool1s[0]; a2.x_elems = (int64_t)B * H * H * 32;
    a2.out_elems = (int64_t)B * (H / 2) * (H / 2) * 64;
    a2.mask[0] = nb.mask2; a2.mask[1] = nullptr;
    M("conv2_fwd");
    CHECK_LAUNCH(pick_tile(kConv2Fwd, H, H).launch(a2, nz, s));
  }
  if (!tower && (!nb.fwd_only || nb.fwd_only == 3)) {
    // conv3 (train_val.prototxt:119-158): split bf16, 8x8 tiles (kConv3Fwd), two k groups
    // of 4 waves; pool3 (= fc4's input) fp32 in Caffe order, routing bytes
    // NHWC (the backward expands dpool3 through them)
    const int H = S / 4;
    SplitArgs a3{};
    a3.B = B; a3.H = H; a3.W = H; a3.pad = 1;
    for (int z = 0; z < 2; ++z) {
      a3.in32[z] = nb.pool2f[z];
      a3.wk[z] = nb.wks[z] + L.wks_off[2];
      a3.bias[z] = nb.theta[z] + L.b[2];
      a3.out[z] = nb.pool3[z];
    }
    a3.xsplit = nb.pool2s[0]; a3.x_elems = (int64_t)B * H * H * 64;   // (conv3's weight gradient)
    a3.wk_elems = L.wks_total;
    a3.nchw = 1;
    a3.mask[0] = nb.mask3; a3.mask[1] = nullptr;
    M("conv3_fwd");
    CHECK_LAUNCH(pick_tile(kConv3Fwd, H, H).launch(a3, nz, s));
  }
  if (nb.fwd_only) return hipSuccess;   // ddq_time_layer: one conv layer
  // fc4 (train_val.prototxt:159-185): split bf16 MFMA register-direct, split-K
  // partials (reduced by the head kernel, or by fc4_reduce_out below)
  const int s4 = S / 8;
  Fc4FwdArgs f;
  f.B = B; f.K = 64 * s4 * s4; f.nz = nz; f.part = nb.fc4_part;
  for (int z = 0; z < 2; ++z) { f.x[z] = nb.pool3[z]; f.w[z] = nb.theta[z] + L.w[3]; }
  M("fc4_fwd");
  CHECK_LAUNCH(launch_fc4_fwd(f, s));
  if (!out) return hipSuccess;   // training: reduce + Q_out fused into the head kernel
  M("fc4_reduce_out");
  ddq_launch(fc4_reduce_out_kernel, dim3(B, nz), dim3(kFc4), 0, s, nb.fc4_part,
                     fc4_fwd_splits(f.K), nz, B, nb.theta[0] + L.b[3], nb.theta[1] + L.b[3],
                     nb.theta[0] + L.w[4], nb.theta[0] + L.b[4], nb.theta[1] + L.w[4],
                     nb.theta[1] + L.b[4], nb.h4[0], nb.h4[1], nb.q_out, nb.p_out);
  CHECK_LAUNCH(hipGetLastError());
  return hipSuccess;
}

hipError_t launch_small_fwd_head(const NetBuffers& nb, hipStream_t s,
                                 void (*mark)(void*, const char*), void* marg, ReplayMeta* bump,
                                 const Prefetch* pf) {
  const ParamLayout& L = nb.L;
  auto M = [&](const char* n) { if (mark) mark(marg, n); };
  // the head's bookkeeping (launch_head / head_args), by K1's extra workgroup
  sm16::BookArgs bk{};
  bk.latch = nb.fa.on ? nb.opt_init : nullptr;
  bk.iter = nb.iter; bk.period = nb.fa.period; bk.inc = nb.book_inc; bk.B = nb.B;
  ReplayMeta* hb = (nb.fa.on || nb.head_bump) ? bump : nullptr;
  if (pf && pf->ng > 0 && hb && nb.B <= 256) {
    bk.dmeta = hb;
    bk.didx = pf->idx; bk.dseed = pf->seed; bk.dlog = pf->idx_log; bk.dlog_cap = pf->log_cap;
  } else {
    bk.bump = hb;
  }
  M("tower_fwd");
  CHECK_LAUNCH(sm16::launch_tower_fwd16(tower_args(nb, 2, &bk), s));
  sm16::ChainArgs c{};
  c.B = nb.B;
  c.x[0] = nb.pool3[0]; c.x[1] = nb.pool3[1];
  c.th[0] = nb.theta[0]; c.th[1] = nb.theta[1];
  c.w4_off = L.w[3]; c.b4_off = L.b[3]; c.w5_off = L.w[4]; c.b5_off = L.b[4];
  if (L.w[3] % 4) return hipErrorInvalidValue;   // (dW4 rows stored as float4)
  c.action = nb.action; c.reward = nb.reward; c.nonterm = nb.nonterm; c.gamma = nb.gamma;
  c.qpart = nb.qpart; c.dpart = nb.dpart; c.sync = nb.csync;
  c.q_out = nb.q_out; c.p_out = nb.p_out; c.q_sa = nb.q_sa; c.p_sa = nb.p_sa;
  c.target = nb.target; c.loss = nb.loss; c.grad = nb.grad;
  c.apply = nb.fa.on && !nb.fa.ext;
  c.store_grad = nb.fa.store_grad;
  c.aa = apply_args(nb, nb.fa.rule, nb.fa.lr, nb.fa.decay, nb.fa.eps, nb.fa.momentum, nb.fa.wd,
                    nb.fa.period);
  c.at = apply_tail(nb);
  c.G = nb.small_G; c.upart = nb.upart; c.w4part = nb.w4part;
  if (c.G > 8 || (c.G > 1 && (!c.upart || !c.w4part))) return hipErrorInvalidValue;
  // B <= 32: one tower a workgroup (kFcBlk of the P tower, then kFcBlk of
  // Q); B > 32: both towers a workgroup, kFcBlk G (all resident)
  const bool one = c.G == 1;
  auto kern = one ? sm16::fc4_chain16_kernel<1> : sm16::fc4_chain16_kernel<2>;
  static std::atomic<uint64_t> attr1{0}, attr2{0};
  CHECK_LAUNCH(ensure_dyn_lds(reinterpret_cast<const void*>(kern), one ? attr1 : attr2,
                              sm16::kChainSmem));
  M("fc4_chain");
  ddq_launch(kern, dim3((one ? 2 : 1) * sm16::kFcBlk * c.G - (nb.fault_k2_short ? 1 : 0)), dim3(512),
             sm16::kChainSmem, s, c);
  CHECK_LAUNCH(hipGetLastError());
  return hipSuccess;
}

void small_groups(int B, int* G2, int* G3) {
  // conv2 tiles: groups of >= 4 images (16 at most: 160 workgroups); conv3
  // tiles: 8 groups of >= 4 images (48 workgroups) -- co-resident with room.
  // (deepq16 B = 32, measured: G2 8 / 16 -> wgrad launch 17.1 / 20.2 us: half
  // the write-through slab bytes, and the meeting's arrival skew with them)
  *G2 = std::max(1, std::min(16, B / 4));
  *G3 = std::max(1, std::min(8, B / 4));
}

// K4's dynamic LDS (launch_small_bwd)
static int wgrad16_lds() {
  // (the staging buffers; the cross-wave sums of a tile's NT accumulators
  // and, with one group, the tile's sums)
  constexpr int NT2 = 5, NT3 = 6;
  return std::max({2 * sm16::Wg2::BUF * 2, 2 * sm16::Wg3::BUF * 2,
                   NT2 * 4 * 16 * 64 * 4 + sm16::Wg2::SLAB * 4,
                   NT3 * 4 * 16 * 64 * 4 + sm16::Wg3::SLAB * 4}) + 16;
}

hipError_t small_coresident(int B, int* ok, char* why, int nwhy) {
  *ok = 1;
  int dev = 0, ncu = 0;
  if (hipError_t e = hipGetDevice(&dev)) return e;
  if (hipError_t e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev)) return e;
  int G2, G3;
  small_groups(B, &G2, &G3);
  const int G = B > 32 ? (B + 31) / 32 : 1;
  struct Launch {
    const char* name;
    const void* kern;
    int threads, lds, meeting;   // meeting: workgroups that wait on each other
  };
  const Launch ls[] = {
      // K1 split form (2 workgroups per (image, tower), B <= 64): pairs meet
      {"tower_fwd16s", reinterpret_cast<const void*>(sm16::tower_fwd16s_kernel<5, 4>),
       sm16::kThreads, sm16::kFwdSmemS, 4 * B <= 256 ? 4 * B : 0},
      // K2: every fc4 workgroup meets (one tower a workgroup at B <= 32)
      {"fc4_chain16", G == 1 ? reinterpret_cast<const void*>(sm16::fc4_chain16_kernel<1>)
                             : reinterpret_cast<const void*>(sm16::fc4_chain16_kernel<2>),
       512, sm16::kChainSmem, (G == 1 ? 2 : 1) * sm16::kFcBlk * G},
      // K4: a tile's groups meet when it has more than one
      {"wgrad16", reinterpret_cast<const void*>(sm16::wgrad16_kernel), 256, wgrad16_lds(),
       (G3 > 1 ? sm16::kT3 * G3 : 0) + (G2 > 1 ? sm16::kT2 * G2 : 0)},
  };
  for (const Launch& l : ls) {
    if (l.meeting == 0) continue;
    if (hipError_t e = hipFuncSetAttribute(l.kern, hipFuncAttributeMaxDynamicSharedMemorySize, l.lds))
      return e;
    int per_cu = 0;
    if (hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, l.kern, l.threads, l.lds))
      return e;
    if ((int64_t)per_cu * ncu < l.meeting) {
      *ok = 0;
      snprintf(why, nwhy, "%s: %d meeting workgroups, %d resident (%d per CU x %d CUs)", l.name,
               l.meeting, per_cu * ncu, per_cu, ncu);
      return hipSuccess;
    }
  }
  return hipSuccess;
}

hipError_t launch_small_bwd(const NetBuffers& nb, hipStream_t s,
                            void (*mark)(void*, const char*), void* marg, bool book,
                            int book_period, ReplayMeta* bump, hipError_t (*fc4_done)(void*),
                            void* fc4_done_arg, const Prefetch* pre) {
  const ParamLayout& L = nb.L;
  const int B = nb.B;
  auto M = [&](const char* n) { if (mark) mark(marg, n); };
  // fc4's weight gradient is final since K2 (B <= 32; else after K4's chunk
  // sums): the overlapped all-reduce starts
  if (fc4_done && nb.small_G == 1) CHECK_LAUNCH(fc4_done(fc4_done_arg));
  {
    sm16::BwdArgs a{};
    a.B = B; a.dpart = nb.dpart;
    a.mask1 = nb.mask1; a.mask2 = nb.mask2; a.mask3 = nb.mask3;
    a.wks = nb.wks[0]; a.wks_plane = L.wks_total; a.wkst_off = L.wkst_off; a.wkst3_off = L.wkst3_off;
    a.frames = nb.state;
    a.dconv3x = nb.dconv3s; a.dconv2x = nb.dconv2x;
    a.w1part = nb.wpart + nb.wpart_off[0]; a.w1_np = nb.wnp[0];
    M("tower_bwd");
    if (2 * B <= 256) {   // split form: two workgroups per image
      constexpr int K3 = 5, KD = 5;   // (KD: tap pairs in flight)
      auto kern = sm16::tower_bwd16s_kernel<K3, KD>;
      static std::atomic<uint64_t> attr{0};
      CHECK_LAUNCH(ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, sm16::kBwdSmem));
      ddq_launch(kern, dim3(2 * B), dim3(sm16::kThreads), sm16::kBwdSmem, s, a);
    } else {
      constexpr int K3 = 5, KD = 6;
      auto kern = sm16::tower_bwd16_kernel<K3, KD>;
      static std::atomic<uint64_t> attr{0};
      CHECK_LAUNCH(ensure_dyn_lds(reinterpret_cast<const void*>(kern), attr, sm16::kBwdSmem));
      ddq_launch(kern, dim3(B), dim3(sm16::kThreads), sm16::kBwdSmem, s, a);
    }
    CHECK_LAUNCH(hipGetLastError());
  }
  {
    sm16::WgArgs w{};
    w.B = B;
    small_groups(B, &w.G2, &w.G3);
    w.ipg2 = (B + w.G2 - 1) / w.G2; w.ipg3 = (B + w.G3 - 1) / w.G3;
    w.pool1s = nb.pool1s[0]; w.pool2s = nb.pool2s[0];
    w.dconv2x = nb.dconv2x; w.dconv3x = nb.dconv3s;
    w.w1part = nb.wpart + nb.wpart_off[0]; w.w1_np = nb.wnp[0];
    w.slab2 = nb.slab2; w.slab3 = nb.slab3;
    w.sync = nb.csync + 8;
    w.poison0 = nb.csync + 2;                  // K2's fan-in
    w.poison1 = nb.csync + 48;                 // K1's pool2 exchange
    w.grad = nb.grad;
    for (int l = 0; l < 3; ++l) { w.w_off[l] = L.w[l]; w.b_off[l] = L.b[l]; }
    conv_dims(L, w.cd);
    w.apply = nb.fa.on && !nb.fa.ext;
    w.aa = apply_args(nb, nb.fa.rule, nb.fa.lr, nb.fa.decay, nb.fa.eps, nb.fa.momentum, nb.fa.wd,
                      nb.fa.period);
    w.at = apply_tail(nb);
    w.book = book; w.book_period = book_period; w.book_inc = nb.book_inc;
    w.iter = nb.iter;
    w.bump = book && !nb.fa.on ? bump : nullptr;
    w.w4_off = L.w[3];
    w.G = nb.small_G; w.upart = nb.upart; w.w4part = nb.w4part;
    w.b4_off = L.b[3]; w.w5_off = L.w[4]; w.b5_off = L.b[4]; w.loss = nb.loss;
    w.nw4 = (w.apply || w.G > 1) ? 32 : 0;
    w.nus = w.G > 1 ? 1 : 0;
    if (L.w[3] % 4) return hipErrorInvalidValue;   // (float4 rows; 94496 for this net)
    if (pre && nb.fa.on) {
      w.pf = *pre;
      w.pf.predrawn = bump != nullptr && B <= 256;   // K1 drew it (its book block)
    }
    // LDS: a round buffer per tile layer, two where a group has more than one
    // round; at least the wave sums + a one-group tile's sums
    const int r2 = (w.ipg2 + sm16::Wg2::NI - 1) / sm16::Wg2::NI;
    const int r3 = (w.ipg3 + sm16::Wg3::NI - 1) / sm16::Wg3::NI;
    (void)r2; (void)r3;   // (two buffers always: the staging's dummy slot follows them)
    const int lds = wgrad16_lds();
    static std::atomic<uint64_t> attr{0};
    CHECK_LAUNCH(ensure_dyn_lds(reinterpret_cast<const void*>(sm16::wgrad16_kernel), attr,
                                sm16::kWgSmem));
    M("wgrad_apply");
    ddq_launch(sm16::wgrad16_kernel,
               dim3(sm16::kT3 * w.G3 + sm16::kT2 * w.G2 + sm16::kW1Blocks + w.pf.ng + w.nw4 +
                    w.nus),
               dim3(256),
               lds, s, w);
    CHECK_LAUNCH(hipGetLastError());
  }
  if (fc4_done && nb.small_G > 1) CHECK_LAUNCH(fc4_done(fc4_done_arg));   // (chunk sums done)
  return hipSuccess;
}

hipError_t launch_backward(const NetBuffers& nb, hipStream_t s, void (*mark)(void*, const char*),
                           void* marg, bool book, int book_period, ReplayMeta* bump,
                           hipError_t (*fc4_done)(void*), void* fc4_done_arg,
                           const Prefetch* pre) {
  const ParamLayout& L = nb.L;
  const int B = nb.B, S = nb.S;
  const int s4 = S / 8;
  auto M = [&](const char* n) { if (mark) mark(marg, n); };
  {  // fc4 (train_val.prototxt:159-185): data gradient -> pooled dpool3, and
     // the weight gradient unless the fused apply computes it itself
    bool narrow;
    int ndx, nd;
    Fc4DgradArgs f = fc4_dgrad_args(nb, narrow, ndx, nd);
    const int nw = (nb.fa.on && !nb.fa.ext) ? 0 : fc4_wgrad_blocks<8>(f.K);
    M("fc4_bwd");
    ddq_launch((narrow ? fc4_bwd_kernel<true, 16> : fc4_bwd_kernel<true, 32>),
                       dim3(nd + nw), dim3(512), 0, s, f, nb.pool3[0], nb.grad + L.w[3], nd, ndx);
    CHECK_LAUNCH(hipGetLastError());
  }
  // the fc4 weight gradient (the bulk of the flat gradient) is final here:
  // the caller may start reducing it over the ranks under the conv backward
  if (fc4_done) CHECK_LAUNCH(fc4_done(fc4_done_arg));
  {  // conv3 data gradient -> split pooled dpool2 (split bf16 on conv3's
     // transposed + flipped split weights, rebuilt by the head kernel; the fp32
     // dpool3 expanded through pool3's routing and split while staged; 4x8 (kConv3Dgrad)
     // tiles x four k groups).  Its staging also writes the expanded split
     // dconv3 (the tiles' own pixels, 16-byte stores) for the weight gradient.
    const int H = S / 4;
    SplitArgs a{};
    a.B = B; a.H = H; a.W = H; a.pad = 1;
    a.in_f32 = nb.dconv3; a.in_route = nb.mask3;
    a.wk[0] = nb.wks[0] + L.wkst3_off; a.wk_elems = L.wks_total;
    a.pd_split = nb.dconv2s; a.pd_elems = (int64_t)B * H * H * 64;
    a.xsplit = nb.dconv3s; a.x_elems = (int64_t)B * H * H * 64;
    M("conv3_dgrad");
    CHECK_LAUNCH(pick_tile(kConv3Dgrad, H, H).launch(a, 1, s));
  }
  {  // conv3 weight gradient (split bf16, wgrads.h): rows of the expanded split
     // dconv3 (pure copies) against the split pool2; conv2's on the split
     // pooled dpool2 and the split pool1
    WgradSArgs w3{}, w2{};
    const int H3 = S / 4, H2 = S / 2;
    w3.B = B; w3.H = H3; w3.W = H3; w3.G = nb.wsplits[2];
    w3.RPG = (B * H3 + w3.G - 1) / w3.G; w3.NP = nb.wnp[2];
    w3.in = nb.pool2s[0]; w3.in_elems = (int64_t)B * H3 * H3 * 64;
    w3.dfull = nb.dconv3s; w3.d_elems = (int64_t)B * H3 * H3 * 64;
    w3.droute = nb.mask3; w3.part = nb.wpart + nb.wpart_off[2];
    w2.B = B; w2.H = H2; w2.W = H2; w2.G = nb.wsplits[1];
    w2.RPG = (B * H2 + w2.G - 1) / w2.G; w2.NP = nb.wnp[1];
    w2.in = nb.pool1s[0]; w2.in_elems = (int64_t)B * H2 * H2 * 32;
    w2.dpool = nb.dconv2s; w2.d_elems = (int64_t)B * (H2 / 2) * (H2 / 2) * 64;
    w2.droute = nb.mask2; w2.part = nb.wpart + nb.wpart_off[1];
    // one launch (wgrads_pair_kernel, conv2's blocks first): 35.2 -> 30.2 us
    // against the two launches, same-box kernel trace
    M("conv23_wgrad");
    CHECK_LAUNCH(launch_wgrads_conv23(w2, w3, s));
  }
  {  // conv2 data gradient -> dpool1 (split bf16, DGRAD): the split pooled
     // dpool2 expanded through mask2 while staged, the transposed split
     // weights the head kernel rebuilt, one 64-channel chunk, 8x16-pixel
     // (kConv2Dgrad) tiles, four k groups (their sums meet in LDS in fixed
     // order) -- and conv1's weight gradient of the tile's conv1 pixels in the
     // same workgroup (split.h w1_tile_wgrad): dpool1 routed through mask1
     // into LDS, the frames' halo, one fp32 slab per tile (train_val.prototxt
     // :39-61; conv1 has no bottom diff)
    const int H = S / 2;
    SplitArgs a{};
    a.B = B; a.H = H; a.W = H; a.pad = 2;
    a.in[0] = nb.dconv2s; a.in_elems = (int64_t)B * (H / 2) * (H / 2) * 64;
    a.wk[0] = nb.wks[0] + L.wkst_off; a.wk_elems = L.wks_total;
    a.in_route = nb.mask2;
    a.w1_route = nb.mask1; a.w1_in = nb.state;
    a.w1_part = nb.wpart + nb.wpart_off[0]; a.w1_np = nb.wnp[0];
    M("conv2_dgrad");
    CHECK_LAUNCH(pick_tile(kConv2Dgrad, H, H).launch(a, 1, s));
  }
  // slab-reduce geometry: layer l's blocks start at d[l].blk0
  WredDims d[3];
  const int cout[3] = {32, 64, 64}, cin[3] = {4, 32, 64}, ks[3] = {7, 5, 3};
  int blk = 0;
  for (int l : {0, 2, 1}) {
    // waves per unit: enough that each holds at most kWredCh slabs (4 at most)
    const int sp = nb.wsplits[l];
    const int G = sp <= kWredCh ? 1 : (sp <= 2 * kWredCh ? 2 : 4);
    d[l] = {L.w[l], L.b[l], nb.wpart_off[l], cout[l], cin[l], ks[l], sp, nb.wnp[l],
            blk, L.wks_off[l], G};
    blk += cout[l] * (nb.wnp[l] / 64) * G / 4;   // units per layer: a multiple of 32
  }
  {  // slab reduce -> grads (Caffe layout) [+ the fused apply + next draw]
    if (nb.fc4_wait) CHECK_LAUNCH(hipStreamWaitEvent(s, nb.fc4_wait, 0));
    M("wgrad_reduce");
    HeadSums hs{0, B, nb.dqbuf, nb.lpart, nb.h4[0], nb.dh4, nb.loss, nb.grad + L.w[4],
                nb.grad + L.b[4], nb.grad + L.b[3]};
    const int nub = blk;
    ApplyTail fat = apply_tail(nb);
    ApplyArgs faa = apply_args(nb, nb.fa.rule, nb.fa.lr, nb.fa.decay, nb.fa.eps, nb.fa.momentum,
                               nb.fa.wd, nb.fa.period);
    int nfa = 0;
    fat.nfa = 0;
    if (nb.fa.on) {   // fc4 weights [w4, b4): its gradient is final since fc4_bwd
      faa.lo = L.w[3];
      faa.hi = L.b[3];
      nfa = fc4_wgrad_blocks<kFc4ApplyR>(64 * s4 * s4);
      fat.nfa = nfa;
      fat.ext = nb.fa.ext;
      fat.store_grad = nb.fa.store_grad;
      // and everything else where its gradient is reduced -- unless the rest
      // must be summed over the ranks first (ext: apply launch after that)
      fat.rest = !nb.fa.ext;
    }
    Prefetch pf{};
    if (pre && nb.fa.on) {
      pf = *pre;
      pf.predrawn = bump != nullptr && nb.B <= 256;   // launch_head drew it (head_draw)
    }
    ddq_launch(wgrad_reduce_kernel, dim3(pf.ng + nub + kFc4 / 64 + nfa), dim3(256), 0, s,
                       nb.wpart, nb.grad, d[0], d[1], d[2], nub, nb.iter,
                       book ? nb.opt_init : nullptr, book_period,
                       book && !nb.fa.on ? bump : nullptr, nb.book_inc, hs, fat, faa, pf,
                       nb.pool3[0], 64 * s4 * s4);
    CHECK_LAUNCH(hipGetLastError());
  }
  return hipSuccess;
}

// ---------------------------------------------------------------------------
// acting: Q forward of n states + argmax (select_action, baristanet.py:142-146)
// ---------------------------------------------------------------------------
__global__ void argmax_kernel(int n, const float* __restrict__ qout, int32_t* __restrict__ actions) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const float* q = qout + b * 4;
  int best = 0;
  for (int a = 1; a < 4; ++a)
    if (q[a] > q[best]) best = a;   // numpy argmax: first max
  actions[b] = best;
}

hipError_t launch_act(const NetBuffers& nb, const float* in, int n, float* pool3, float* h4,
                      float* part, float* qout, int32_t* actions, __bf16* pool1s,
                      __bf16* pool2s, hipStream_t s) {
  NetBuffers a = nb;
  a.B = n;
  a.state = const_cast<float*>(in);
  a.next_state = const_cast<float*>(in);
  a.pool3[0] = pool3; a.h4[0] = h4;
  a.pool3[1] = pool3; a.h4[1] = h4;
  // (no weight gradient: no split side outputs; the scratch holds fp32)
  a.pool1s[0] = a.pool1s[1] = nullptr; a.pool2s[0] = a.pool2s[1] = nullptr;
  a.pool1f[0] = a.pool1f[1] = reinterpret_cast<float*>(pool1s);
  a.pool2f[0] = a.pool2f[1] = reinterpret_cast<float*>(pool2s);
  a.mask1 = a.mask2 = a.mask3 = nullptr;
  a.fc4_part = part;
  a.q_out = qout; a.p_out = qout;
  CHECK_LAUNCH(launch_forward(a, 1, s, nullptr, nullptr));
  if (actions) {
    ddq_launch(argmax_kernel, dim3((n + 63) / 64), dim3(64), 0, s, n, qout, actions);
    CHECK_LAUNCH(hipGetLastError());
  }
  return hipSuccess;
}

}  // namespace ddq
