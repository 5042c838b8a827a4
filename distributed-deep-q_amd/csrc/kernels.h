// Host-side launch wrappers for the deepq step kernels (implemented in
// kernels.hip).  All launches are asynchronous on the given stream and
// graph-capture safe (no allocation, no synchronisation).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"   // ddq_launch / ExtTiming (kernel timing)

namespace ddq {

// Flat parameter layout of one tower (pycaffe order), element offsets.
struct ParamLayout {
  int S, S2, S3, S4;
  int64_t w[5], b[5];      // offsets of layer weights / biases
  int64_t wn[5], bn[5];    // counts
  int64_t total;
  int64_t wks_off[3];      // offsets of the split (3 x bf16) forward weights in a wks plane
  int64_t wkst_off;        // conv2 data-gradient split weights [ci][tap'][co] (Q only)
  int64_t wkst3_off;       // conv3 data-gradient split weights [ci][tap'][co] (Q only)
  int64_t wks_total;       // elements per wks plane (conv1 padded to kx = 8)
};
ParamLayout make_layout(int S);

// Replay ring bookkeeping kept in device memory so captured graphs see the
// live head/valid and a fresh RNG counter on every replay.
struct ReplayMeta {
  int64_t head, valid, capacity;
  uint64_t counter;        // device index-stream draws so far
  int32_t err;             // sticky: 1 = stored action >= num_actions seen,
                           //         2 = a draw found no distinct index set
  int32_t pad;
};

// Fused apply: the update rule of the step.  ext = 0 (exchange-free steps):
// the slab-reduce launch computes fc4's weight gradient tile by tile and
// updates every parameter where its gradient becomes final.  ext = 1 (RCCL
// all-reduce with overlap): fc4_bwd computes fc4's weight gradient, the comm
// stream sums it over the ranks under the conv backward (fc4_wait), the
// slab-reduce launch applies fc4's weights from it, and launch_apply the rest
// after their (small) all-reduce.
struct FusedApplyCfg {
  int on, ext;
  int store_grad;             // fc4's weight gradient also to the gradient buffer
  int rule, period;
  float lr, decay, eps, momentum, wd;
};

struct Prefetch;

struct NetBuffers {
  int B, S;
  // minibatch (NHWC frames; action one-hot (B,4); reward / non_terminal (B))
  float *state, *next_state, *action, *reward, *nonterm;
  int32_t* idx;
  // activations per tower z (0 = Q on state, 1 = P on next_state): pool1 /
  // pool2 in one buffer each, sized for their split form (3 bf16 planes,
  // NHWC) -- the S = 16 small-map step keeps the Q tower's split there (its K4
  // reads them split); the general kernels keep fp32 NHWC in the same bytes
  // (pool1f / pool2f: the next conv and the Q weight gradients split them
  // while staging); pool3 fp32 in Caffe order (fc4's input)
  float *pool3[2], *h4[2];
  __bf16 *pool1s[2], *pool2s[2];    // split pool1 / pool2 (3 planes, NHWC): small-map step
  float *pool1f[2], *pool2f[2];     // the same bytes, fp32 NHWC: general kernels
  uint8_t *mask1, *mask2, *mask3;   // Q tower only
  float* fc4_part;                  // [splits][2][B][512]
  int fc4_splits;
  // optional device index log: draw d's sorted indices at [(d % log_cap) * B]
  int32_t* idx_log;
  int64_t log_cap;
  // blobs
  float *q_out, *p_out, *q_sa, *p_sa, *target, *loss;
  // backward scratch
  float *dh4, *dconv3;               // dh4 (B,512); dconv3: fp32 pooled dpool3 (fc4 dgrad)
  __bf16* dconv2s;                  // split pooled dpool2 (conv3's data gradient)
  __bf16* dconv3s;                  // split expanded dconv3 (B,S/4,S/4,64): conv3's weight gradient
  float* wpart;                     // conv wgrad slabs (3 layers, disjoint)
  int64_t wpart_off[3];
  int wsplits[3];
  int wnp[3];
  // parameters: theta[z] flat Caffe layout; wks[z] split kernel layouts (the
  // forward convs; Q's also the data gradients' transposed copies); grad; opt
  // state
  float *theta[2], *grad, *opt;
  __bf16* wks[2];
  float *dqbuf, *lpart;             // head: per-sample dQ (B,4) and squared error (B)
  int32_t* opt_init;                // 0 until the first apply after a reset
  int64_t* iter;                    // applied updates (param-server iteration)
  // side stream + events: the next step's sample + gather beside a step whose
  // apply launch cannot carry them (pipelined stepping, B > 256)
  hipStream_t side;
  hipEvent_t ev[8];
  hipEvent_t fc4_wait;              // the slab-reduce launch waits for it (fa.ext)
  ParamLayout L;
  float gamma;
  int fwd_only;                     // launch_forward: 0 = every layer, l + 1 = conv layer l only
  int fault_k2_short = 0;           // ddq_inject_fault (tests): this step's fc4 chain launch
                                    // one workgroup short, so its fan-in meeting times out
  FusedApplyCfg fa;                 // on: head latches the apply flags, the slab reduce
                                    // applies (FusedApplyCfg)
  int book_inc;                     // param-server iterations per apply (1, or W: server mode)
  int head_bump;                    // the head kernel advances the draw counter without a
                                    // fused apply (async gradients: sample_gather draws)
  // deepq16 step (small.h, small_bwd.h): fc4 chain partials and its fan-in words
  int small;                        // S == 16, B <= 256: the four-launch step
  int small_G = 1;                  // its fc4 chain's image chunks (B > 32: ceil(B / 32))
  float* upart = nullptr;           // [G][32][96] unit-sum partials (G > 1)
  float* w4part = nullptr;          // [G][512][256] fc4 weight-gradient partials (G > 1)
  float *qpart, *dpart;             // [32][2][B][4] Q_out / P_out partials, [32][B][256] dpool3
  int32_t* csync;                   // meeting words: K2 [0..2] (64-bit counter, timeout),
                                    // K4 [8..40) (a 64-bit counter per tile, timeout at
                                    // 40), K1's split form: timeout at 48
  __bf16* dconv2x;                  // split expanded dconv2 NHWC (B, 8, 8, 64) (K3 -> K4)
  float *slab2, *slab3;             // K4's per-group slabs of conv2 / conv3 tiles
  __bf16* xchg;                     // K1 split form: pool2 halves [B][2][2][1536]
  uint64_t* pairc;                  // K1 split form: meeting counters [B][2]
};

// fused device draw + gather for the step (B <= 256); counter advanced by the
// step's apply bookkeeping (launch_backward's bump)
hipError_t launch_sample_gather(const NetBuffers& nb, const uint8_t* st, const uint8_t* act,
                                const int16_t* rew, const uint8_t* nt, ReplayMeta* meta,
                                uint64_t seed, hipStream_t s);
hipError_t launch_gather(const NetBuffers& nb, const uint8_t* st, const uint8_t* act,
                         const int16_t* rew, const uint8_t* nt, ReplayMeta* meta,
                         hipStream_t s);
hipError_t launch_sample(const NetBuffers& nb, ReplayMeta* meta, uint64_t seed, hipStream_t s);
hipError_t launch_forward(const NetBuffers& nb, int nz, hipStream_t s, void (*mark)(void*, const char*), void* mark_arg,
                          bool out = true);
// deepq16 (nb.small): K1 (towers + the head's bookkeeping: latch, bump /
// next draw, as launch_head's) and K2 (fc4 chain) in place of launch_forward
// + launch_head
// Every meeting launch of the small-map step has all of its meeting
// workgroups resident at once on this device (meet() spins on the others):
// *ok = 0 and why set otherwise (the ctx then runs the general kernels)
hipError_t small_coresident(int B, int* ok, char* why, int nwhy);
hipError_t launch_small_fwd_head(const NetBuffers& nb, hipStream_t s,
                                 void (*mark)(void*, const char*), void* mark_arg,
                                 ReplayMeta* bump = nullptr, const struct Prefetch* pf = nullptr);
// bump (fused apply only): the step's draw-counter advance, done here so the
// slab-reduce launch can carry the next step's draw + gather
hipError_t launch_head(const NetBuffers& nb, hipStream_t s, ReplayMeta* bump = nullptr,
                       const Prefetch* pf = nullptr);
bool fused_apply_ok(const ParamLayout& L);
// book: the slab reduce also does the apply bookkeeping (target period
// book_period); fc4_done: called right after the fc4 weight gradient is
// enqueued (the overlapped all-reduce starts there); pf (fused apply only):
// the next step's draw + gather as blocks of the slab-reduce launch.
// deepq16 (nb.small): K3 (data gradients, conv1's weight gradient slabs)
// and K4 (conv weight gradients + fused apply + bookkeeping + next gather) in
// place of launch_backward (same arguments)
hipError_t launch_small_bwd(const NetBuffers& nb, hipStream_t s, void (*mark)(void*, const char*),
                            void* mark_arg, bool book, int book_period, ReplayMeta* bump,
                            hipError_t (*fc4_done)(void*), void* fc4_done_arg,
                            const struct Prefetch* pf);
void small_groups(int B, int* G2, int* G3);
hipError_t launch_backward(const NetBuffers& nb, hipStream_t s, void (*mark)(void*, const char*),
                           void* mark_arg, bool book = false, int book_period = 0,
                           ReplayMeta* bump = nullptr, hipError_t (*fc4_done)(void*) = nullptr,
                           void* fc4_done_arg = nullptr, const Prefetch* pf = nullptr);
// period > 0: also copy Q -> P when the next pull sees iteration % period == 0.
// Next step's draw + gather carried by the apply launch (pipelined stepping)
struct Prefetch {
  const uint8_t* st;
  const uint8_t* act;
  const int16_t* rew;
  const uint8_t* nt;
  ReplayMeta* meta;
  uint64_t seed;
  int B, S, gx, ng;                 // ng = 0: no prefetch blocks
  int predrawn;                     // 1: the head launch drew the set into idx already
  int32_t* idx;
  int32_t* idx_log;                 // NetBuffers::idx_log / log_cap of the step
  int64_t log_cap;
  float *sQ, *sP, *action, *reward, *nonterm;
};
Prefetch make_prefetch(const NetBuffers& next, const uint8_t* st, const uint8_t* act,
                       const int16_t* rew, const uint8_t* nt, ReplayMeta* meta, uint64_t seed);
hipError_t launch_apply(const NetBuffers& nb, int rule, float lr, float decay, float eps,
                        float momentum, float wd, int period, bool booked, hipStream_t s,
                        const Prefetch* pre = nullptr);
hipError_t launch_relayout(const NetBuffers& nb, int z, hipStream_t s);
// owner apply of shard [off, off+len) with W gradient slices (stride `slice`)
// applied in rank order; then, after the theta all-gather, launch_refresh
// rebuilds the conv kernel layouts and performs a latched P <- Q sync.
// theta: the parameters updated (default nb.theta[0]; the async exchange's
// owner copy otherwise).  first >= 0: the rules' first-call flag from the host
// and the apply's bookkeeping (iteration += 1) done by the launch itself
// (async owner applies); -1: the flags latched by a prior launch_book.
// pre: the next step's draw + gather as extra blocks (pipelined steps)
// refresh_own != 0: the launch also does launch_refresh's work for its own
// shard (conv kernel layouts of nb.wks[0]; the P <- Q copy into nb.theta[1] /
// nb.wks[1] when a sync is due: -1 the latched flag decides, 1 no sync, 2
// sync), from the values it applied; the refresh after the all-gather / pull
// then skips that shard.  own_g: slice own_w
// is read from there (the rank's own gradient in place) instead of gsl
hipError_t launch_apply_shard(const NetBuffers& nb, int rule, float lr, float decay, float eps,
                              float momentum, float wd, const float* gsl, int64_t off,
                              int64_t len, int64_t slice, int W, hipStream_t s,
                              float* theta = nullptr, int first = -1,
                              const Prefetch* pre = nullptr, float* mirror = nullptr,
                              int refresh_own = 0, int own_w = -1,
                              const float* own_g = nullptr);
// force_sync >= 0: P <- Q decided by the host instead of the latched flag.
// [skip_lo, skip_hi): a range already refreshed (an owner's refresh_own
// apply); nothing is launched when it covers every parameter
hipError_t launch_refresh(const NetBuffers& nb, hipStream_t s, int force_sync = -1,
                          int64_t skip_lo = 0, int64_t skip_hi = 0);
// one apply's bookkeeping (first-call / sync latches, iteration += 1)
hipError_t launch_book(const NetBuffers& nb, int period, hipStream_t s);
hipError_t launch_sum_slices(float* out, const float* in, int W, int64_t len, int64_t slice,
                             hipStream_t s);
// Q-tower forward of n states (NHWC f32 in `in`) into scratch, argmax into out.
hipError_t launch_act(const NetBuffers& nb, const float* in, int n, float* pool3, float* h4,
                      float* part, float* qout, int32_t* actions, __bf16* pool1s,
                      __bf16* pool2s, hipStream_t s);
// large-batch device draw (bitmap claim + ordered compaction) into idx[0..n)
// and the Caffe-layout (n,4,S,S) f32 gather of replay.py:167-183
hipError_t launch_sample_batch(ReplayMeta* meta, int64_t valid, int n, uint64_t seed,
                               uint64_t ctr, uint32_t* bm, int32_t* blk, int32_t* idx,
                               hipStream_t s);
hipError_t launch_gather_nchw(const uint8_t* st, const uint8_t* act, const int16_t* rew,
                              const uint8_t* nt, ReplayMeta* meta, const int32_t* idx, int n,
                              int S, float* s0, float* s1, float* action, float* reward,
                              float* nonterm, hipStream_t s);
hipError_t launch_tile(uint8_t* dst, const uint8_t* src, uint64_t pool_bytes, uint64_t total,
                       hipStream_t s);
hipError_t launch_u8_to_nhwc(const uint8_t* src, int n, int S, float* dst, hipStream_t s);

double step_flops(int B, int S);

extern thread_local const char* g_launch_where;

}  // namespace ddq
