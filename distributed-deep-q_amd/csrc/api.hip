// libddq_hip C-ABI (include/ddq_hip.h): context, device memory, replay ring,
// step orchestration, hipGraph capture, RCCL gradient exchange.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ddq_hip.h"
#include "kernels.h"

namespace ddq {
int fc4_splits_for(int S);
int wgrad_splits_for(int layer, int B, int S, int* np);
}  // namespace ddq

using namespace ddq;

static thread_local std::string g_last_error;

static constexpr int kMaxRanks = 64;
static constexpr int64_t kShardPad = 64 * kMaxRanks;

struct ddq_ctx {
  int device = 0;
  ddq_net_desc desc{};
  hipStream_t stream = nullptr;
  bool own_stream = true;
  NetBuffers nb{};
  std::vector<void*> allocs;
  std::string err;
  // replay ring
  uint8_t* r_state = nullptr;
  uint8_t* r_action = nullptr;
  int16_t* r_reward = nullptr;
  uint8_t* r_nonterm = nullptr;
  ReplayMeta* r_meta = nullptr;    // device
  uint32_t* r_bitmap = nullptr;    // large-batch sampler scratch (lazy)
  int32_t* r_blk = nullptr;
  uint64_t batch_ctr = 0;          // large-batch draws so far (RNG stream position)
  int64_t head = 0, valid = 0, capacity = 0;
  // acting scratch
  uint8_t* act_u8 = nullptr;
  float *act_in = nullptr, *act_p3 = nullptr;
  float *act_h4 = nullptr, *act_part = nullptr, *act_q = nullptr;
  __bf16 *act_p1s = nullptr, *act_p2s = nullptr;
  int32_t* act_out = nullptr;
  // index log (ddq_index_log_enable)
  int32_t* log_buf = nullptr;
  int64_t log_buf_cap = 0;
  int64_t log_first = 0;           // first draw the log holds (the counter at enable)
  // comm (RCCL ranks, or an in-process group of ctxs exchanging by device copies)
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  bool local = false;              // member of an in-process group (ddq_group_init)
  hipStream_t cs = nullptr;        // comm stream of the overlapped all-reduce
  hipEvent_t cev[3] = {};
  int64_t shard_len = 0;           // parameters owned per rank (multiple of 64)
  float* gsl = nullptr;            // [W][shard_len] received gradient slices
  float* gstage = nullptr;         // [W][P] in-process all-reduce staging
  // async exchange: the central model's shard this rank owns (Q, and P as of
  // the last special-update pull), both at full-vector offsets
  float* own = nullptr;
  float* pown = nullptr;
  bool async_on = false;           // the async exchange began (async_begin)
  std::vector<int64_t> last_pull;  // iteration of every worker's last pull
  int64_t async_ticks = 0;         // pushes applied since async_begin
  hipEvent_t grad_ev = nullptr;    // this worker's gradient is ready (pushable)
  hipEvent_t tick_ev = nullptr;    // owner duties of the last tick done (comm stream)
  int64_t straggle_us = 0;         // ddq_set_straggle: host-side delay per gradient
  bool ready_seen = false;         // grad_ev observed complete at ready_at
  std::chrono::steady_clock::time_point ready_at{};
  int64_t rr_rounds = 0;           // round-robin rounds since the last ticket-order tick
  bool acapture = false;           // capturing async rounds: grad_ev recorded before the
  bool grad_ev_captured = false;   // capture began is not waited on (the graph launch
                                   // follows that work on the stream anyway)
  hipGraphExec_t agexec = nullptr; // kAsync round-robin rounds as one graph
  int agraph_rounds = 0;
  int64_t agraph_phase = -1;       // iteration % period the graph was captured at
  ddq_step_cfg acfg{};
  // ticket-order ticks of this rank's own gradient as graphs, one per (P pull
  // due, special update due): ddq_async_tick replays instead of re-enqueueing
  hipGraphExec_t tgexec[4] = {nullptr, nullptr, nullptr, nullptr};
  ddq_step_cfg tcfg{};
  std::string comm_err;
  // ddq_inject_fault: armed failpoint, consumed by the next eager step
  int fault = 0;
  std::string small_off;           // why the small-map step is off at S = 16 (empty: on)
  // graph
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec = nullptr;     // one step
  hipGraphExec_t gexec_k = nullptr;   // kGraphSteps steps
  ddq_step_cfg gcfg{};
  bool have_graph = false;
  // pipelined stepping: a second minibatch set and graphs [parity][prefetch]
  float *mb2_state = nullptr, *mb2_next = nullptr, *mb2_action = nullptr;
  float *mb2_reward = nullptr, *mb2_nonterm = nullptr;
  int32_t* mb2_idx = nullptr;
  hipGraphExec_t pexec[2][2] = {};  // one step on set p, [f] = prefetching
  hipGraphExec_t pexec_k[2] = {};   // kGraphSteps prefetching steps starting on set p
  hipGraphExec_t ptail[2][9] = {};  // r = 1..kGraphSteps steps from set p, the last one
                                    // not prefetching (the end of a fused chain)
  ddq_step_cfg pcfg{};
  bool have_pipe = false;
  int64_t steps = 0;
  int64_t applied = 0;               // host mirror of the device iteration counter
  // profiling marks: a kernel's own dispatch start / stop events
  struct Mark {
    std::string name;
    hipEvent_t start, stop;
  };
  std::vector<Mark> marks;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
};

static int fail(ddq_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  g_last_error = buf;
  return code;
}

#define HIP_TRY(c, x)                                                                         \
  do {                                                                                        \
    g_launch_where = "";                                                                      \
    (void)hipGetLastError();  /* launches report via hipGetLastError: drop stale errors */    \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess)                                                                     \
      return fail((c), DDQ_EHIP, "%s failed: %s (%s:%d%s%s)", #x, hipGetErrorString(e_),      \
                  __FILE__, __LINE__, *g_launch_where ? ", at " : "", g_launch_where);        \
  } while (0)

#define NCCL_TRY(c, x)                                                                           \
  do {                                                                                           \
    ncclResult_t r_ = (x);                                                                       \
    if (r_ != ncclSuccess) return fail((c), DDQ_ERCCL, "%s failed: %s", #x, ncclGetErrorString(r_)); \
  } while (0)

template <class T>
static int dalloc(ddq_ctx* c, T** p, size_t count) {
  void* q = nullptr;
  const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess) return fail(c, DDQ_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
  // stream-ordered zero fill: every device access of the ctx goes through
  // c->stream (a non-blocking stream does not order against the null stream)
  e = hipMemsetAsync(q, 0, bytes, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipMemsetAsync failed: %s", hipGetErrorString(e));
  c->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return DDQ_OK;
}

#define TRY(x)                \
  do {                        \
    int r_ = (x);             \
    if (r_ != DDQ_OK) return r_; \
  } while (0)

// Blocking copy ordered on the ctx stream.
static hipError_t scopy(ddq_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, c->stream);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(c->stream);
}

static int set_dev(ddq_ctx* c) {
  HIP_TRY(c, hipSetDevice(c->device));
  return DDQ_OK;
}

static void invalidate_graph(ddq_ctx* c) {
  // (the async tick / round graphs too: they bake in the index log and the
  // other captured pointers that ddq_index_log_enable / set_stream replace)
  for (auto& g : c->tgexec) {
    if (g) hipGraphExecDestroy(g);
    g = nullptr;
  }
  if (c->agexec) hipGraphExecDestroy(c->agexec);
  c->agexec = nullptr;
  c->agraph_rounds = 0;
  if (c->gexec) hipGraphExecDestroy(c->gexec);
  if (c->gexec_k) hipGraphExecDestroy(c->gexec_k);
  c->gexec_k = nullptr;
  if (c->graph) hipGraphDestroy(c->graph);
  c->gexec = nullptr;
  c->graph = nullptr;
  c->have_graph = false;
  for (auto& row : c->pexec)
    for (auto& g : row) {
      if (g) hipGraphExecDestroy(g);
      g = nullptr;
    }
  for (auto& g : c->pexec_k) {
    if (g) hipGraphExecDestroy(g);
    g = nullptr;
  }
  for (auto& row : c->ptail)
    for (auto& g : row) {
      if (g) hipGraphExecDestroy(g);
      g = nullptr;
    }
  c->have_pipe = false;
}

extern "C" {

int ddq_abi_version(void) { return DDQ_ABI_VERSION; }

const char* ddq_last_error(const ddq_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_last_error.c_str();
}

int ddq_create(ddq_ctx** out, int device, const ddq_net_desc* desc) {
  if (!out || !desc) return fail(nullptr, DDQ_EINVAL, "null argument");
  *out = nullptr;
  if (desc->channels != 4 || desc->actions != 4)
    return fail(nullptr, DDQ_EINVAL, "channels and actions must be 4 (got %d, %d)",
                desc->channels, desc->actions);
  if (desc->frame < 16 || desc->frame % 8 != 0 || desc->frame > 1024)
    return fail(nullptr, DDQ_EINVAL, "frame side must be a multiple of 8 in [16,1024] (got %d)",
                desc->frame);
  if (desc->batch < 1 || desc->batch > 1024)
    return fail(nullptr, DDQ_EINVAL, "batch must be in [1,1024] (got %d)", desc->batch);
  // the kernels address every tensor through 32-bit buffer descriptors /
  // offsets (kOOB = 2^31 marks an out-of-range vector): the largest ones are
  // a split activation plane (16 B S^2 bytes) and fc4's weights (2^11 S^2)
  if ((int64_t)16 * desc->batch * desc->frame * desc->frame >= (1ll << 31) ||
      (int64_t)2048 * desc->frame * desc->frame >= (1ll << 31))
    return fail(nullptr, DDQ_EINVAL,
                "batch * frame^2 too large for 32-bit tensor offsets (need 16*B*S^2 < 2^31 "
                "and S < 1024; got B=%d, S=%d)", desc->batch, desc->frame);
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return fail(nullptr, DDQ_EHIP, "no HIP device available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= ndev)
    return fail(nullptr, DDQ_EINVAL, "device %d out of range (%d devices)", device, ndev);
  ddq_ctx* c = new ddq_ctx();
  c->device = device;
  c->desc = *desc;
  int rc = [&]() -> int {
    TRY(set_dev(c));
    HIP_TRY(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    NetBuffers& nb = c->nb;
    HIP_TRY(c, hipStreamCreateWithFlags(&nb.side, hipStreamNonBlocking));
    for (auto& e : nb.ev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const int B = desc->batch, S = desc->frame;
    nb.B = B; nb.S = S; nb.gamma = desc->gamma;
    nb.L = make_layout(S);
    const int64_t P = nb.L.total;
    const int S2 = S / 2, S3 = S / 4, S4 = S / 8;
    TRY(dalloc(c, &nb.state, (size_t)B * S * S * 4));
    TRY(dalloc(c, &nb.next_state, (size_t)B * S * S * 4));
    TRY(dalloc(c, &nb.action, (size_t)B * 4));
    TRY(dalloc(c, &nb.reward, (size_t)B));
    TRY(dalloc(c, &nb.nonterm, (size_t)B));
    TRY(dalloc(c, &nb.idx, (size_t)B));
    for (int z = 0; z < 2; ++z) {
      TRY(dalloc(c, &nb.pool3[z], (size_t)B * S4 * S4 * 64));
      TRY(dalloc(c, &nb.h4[z], (size_t)B * 512));
      TRY(dalloc(c, &nb.theta[z], (size_t)P + kShardPad));
      TRY(dalloc(c, &nb.wks[z], (size_t)3 * nb.L.wks_total));   // zero: conv1's kx 7 stays 0
      TRY(dalloc(c, &nb.pool1f[z], (size_t)B * S2 * S2 * 32));
      TRY(dalloc(c, &nb.pool2f[z], (size_t)B * S3 * S3 * 64));
    }
    TRY(dalloc(c, &nb.pool1s[0], (size_t)3 * B * S2 * S2 * 32));   // Q tower only
    TRY(dalloc(c, &nb.pool2s[0], (size_t)3 * B * S3 * S3 * 64));
    TRY(dalloc(c, &nb.mask1, (size_t)B * S2 * S2 * 32));
    TRY(dalloc(c, &nb.mask2, (size_t)B * S3 * S3 * 64));
    TRY(dalloc(c, &nb.mask3, (size_t)B * S4 * S4 * 64));
    nb.fc4_splits = fc4_splits_for(S);
    TRY(dalloc(c, &nb.fc4_part, (size_t)nb.fc4_splits * 2 * B * 512));
    TRY(dalloc(c, &nb.q_out, (size_t)B * 4));
    TRY(dalloc(c, &nb.p_out, (size_t)B * 4));
    TRY(dalloc(c, &nb.q_sa, (size_t)B));
    TRY(dalloc(c, &nb.p_sa, (size_t)B));
    TRY(dalloc(c, &nb.target, (size_t)B));
    TRY(dalloc(c, &nb.loss, 1));
    TRY(dalloc(c, &nb.dh4, (size_t)B * 512));
    TRY(dalloc(c, &nb.dqbuf, (size_t)B * 4));
    TRY(dalloc(c, &nb.lpart, (size_t)B));
    TRY(dalloc(c, &nb.dconv3, (size_t)B * S3 * S3 * 64));
    TRY(dalloc(c, &nb.dconv2s, (size_t)3 * B * S3 * S3 * 64));
    TRY(dalloc(c, &nb.dconv3s, (size_t)3 * B * S3 * S3 * 64));
    if (S == 16) {   // K1 (tower_fwd16s): the pool2 halves' exchange; meeting words
      TRY(dalloc(c, &nb.xchg, (size_t)B * 2 * 2 * 1536));
      TRY(dalloc(c, &nb.pairc, (size_t)B * 2));
      TRY(dalloc(c, &nb.csync, 64));
    }
    // the four-launch small-map step needs every meeting launch's workgroups
    // co-resident (small_coresident); otherwise the general kernels run
    nb.small = 0;
    if (S == 16 && B <= 256) {
      int ok = 0;
      char why[256] = "";
      HIP_TRY(c, small_coresident(B, &ok, why, sizeof(why)));
      nb.small = ok;
      if (!ok) c->small_off = why;
    } else {
      c->small_off = S == 16 ? "batch > 256" : "frame != 16";
    }
    if (nb.small) {
      TRY(dalloc(c, &nb.qpart, (size_t)32 * 2 * B * 4));
      TRY(dalloc(c, &nb.dpart, (size_t)32 * B * 256));
      TRY(dalloc(c, &nb.dconv2x, (size_t)3 * B * 4096));
      int G2, G3;
      small_groups(B, &G2, &G3);
      TRY(dalloc(c, &nb.slab2, (size_t)10 * G2 * (32 * 5 * 32 + 32)));
      TRY(dalloc(c, &nb.slab3, (size_t)6 * G3 * (32 * 3 * 64 + 32)));
      nb.small_G = B > 32 ? (B + 31) / 32 : 1;   // <= 8: 32 G fc4 workgroups, all resident
      if (nb.small_G > 1) {
        TRY(dalloc(c, &nb.upart, (size_t)nb.small_G * 32 * 96));
        TRY(dalloc(c, &nb.w4part, (size_t)nb.small_G * 512 * 256));
      }
    }
    int64_t off = 0;
    const int cout[3] = {32, 64, 64};
    for (int l = 0; l < 3; ++l) {
      nb.wsplits[l] = wgrad_splits_for(l, B, S, &nb.wnp[l]);
      nb.wpart_off[l] = off;
      off += (int64_t)nb.wsplits[l] * cout[l] * nb.wnp[l];
    }
    TRY(dalloc(c, &nb.wpart, (size_t)off));
    // zero tails of kShardPad floats: W equal shards of a multiple of 64
    // floats cover P for every W <= kMaxRanks
    TRY(dalloc(c, &nb.grad, (size_t)P + kShardPad));
    TRY(dalloc(c, &nb.opt, (size_t)P + kShardPad));
    nb.book_inc = 1;
    TRY(dalloc(c, &nb.opt_init, 4));
    TRY(dalloc(c, &nb.iter, 1));
    // acting scratch (n <= B)
    TRY(dalloc(c, &c->act_u8, (size_t)B * 4 * S * S));
    TRY(dalloc(c, &c->act_in, (size_t)B * S * S * 4));
    TRY(dalloc(c, &c->act_p1s, (size_t)3 * B * S2 * S2 * 32));
    TRY(dalloc(c, &c->act_p2s, (size_t)3 * B * S3 * S3 * 64));
    TRY(dalloc(c, &c->act_p3, (size_t)B * S4 * S4 * 64));
    TRY(dalloc(c, &c->act_h4, (size_t)B * 512));
    TRY(dalloc(c, &c->act_part, (size_t)nb.fc4_splits * 2 * B * 512));
    TRY(dalloc(c, &c->act_q, (size_t)B * 4));
    TRY(dalloc(c, &c->act_out, (size_t)B));
    TRY(dalloc(c, &c->r_meta, 1));
    return DDQ_OK;
  }();
  if (rc != DDQ_OK) {
    g_last_error = c->err;
    ddq_destroy(c);
    return rc;
  }
  *out = c;
  return DDQ_OK;
}

int ddq_destroy(ddq_ctx* c) {
  if (!c) return DDQ_OK;
  hipSetDevice(c->device);
  if (c->cs) hipStreamSynchronize(c->cs);
  if (c->stream) hipStreamSynchronize(c->stream);
  invalidate_graph(c);   // (every graph exec: the step, pipelined, async ones)
  for (auto& e : c->ev_pool) hipEventDestroy(e);
  if (c->comm) ncclCommDestroy(c->comm);
  for (void* p : c->allocs) hipFree(p);
  if (c->stream && c->own_stream) hipStreamDestroy(c->stream);
  for (auto& e : c->nb.ev)
    if (e) hipEventDestroy(e);
  if (c->nb.side) hipStreamDestroy(c->nb.side);
  if (c->cs) hipStreamDestroy(c->cs);
  if (c->grad_ev) hipEventDestroy(c->grad_ev);
  if (c->tick_ev) hipEventDestroy(c->tick_ev);
  for (auto& e : c->cev)
    if (e) hipEventDestroy(e);
  delete c;
  return DDQ_OK;
}

int ddq_set_stream(ddq_ctx* c, void* s) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->own_stream) hipStreamDestroy(c->stream);
  if (s) {
    c->stream = reinterpret_cast<hipStream_t>(s);
    c->own_stream = false;
  } else {
    HIP_TRY(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  invalidate_graph(c);
  return DDQ_OK;
}

int ddq_get_stream(const ddq_ctx* c, void** s) {
  if (!c || !s) return fail(nullptr, DDQ_EINVAL, "null argument");
  *s = reinterpret_cast<void*>(c->stream);
  return DDQ_OK;
}

int ddq_synchronize(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  if (c->cs) HIP_TRY(c, hipStreamSynchronize(c->cs));   // owner duties of async ticks
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (c->nb.csync) {                  // the small-map kernels' sticky spin-timeout words
    int32_t w[64];
    HIP_TRY(c, hipMemcpy(w, c->nb.csync, sizeof(w), hipMemcpyDeviceToHost));
    const int at[3] = {2, 40, 48};
    const char* who[3] = {"fc4 chain fan-in", "wgrad slab reduce", "tower pool2 exchange"};
    for (int k = 0; k < 3; ++k)
      if (w[at[k]]) {
        // the launches after the failure wrote no parameter, optimizer state
        // or iteration (they read the sticky words); start the meeting
        // counters afresh (a launch short of a party leaves them off by its
        // count) and take the device iteration back as the host's
        HIP_TRY(c, hipMemsetAsync(c->nb.csync, 0, 64 * sizeof(int32_t), c->stream));
        if (c->nb.pairc)
          HIP_TRY(c, hipMemsetAsync(c->nb.pairc, 0, (size_t)c->nb.B * 2 * sizeof(uint64_t), c->stream));
        int64_t it = 0;
        HIP_TRY(c, hipMemcpyAsync(&it, c->nb.iter, sizeof(it), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->applied = it;
        return fail(c, DDQ_ESTATE,
                    "small-map step: %s meeting timed out (that step and any after it up to "
                    "this call applied nothing)", who[k]);
      }
  }
  return DDQ_OK;
}

int ddq_inject_fault(ddq_ctx* c, int32_t fault) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (fault == DDQ_FAULT_NONE) {
    c->fault = 0;
    return DDQ_OK;
  }
  if (fault != DDQ_FAULT_MEET_TIMEOUT) return fail(c, DDQ_EINVAL, "unknown fault %d", fault);
  if (!c->nb.small) return fail(c, DDQ_ESTATE, "no small-map step on this ctx (S = 16, B <= 256)");
  c->fault = fault;
  return DDQ_OK;
}

int ddq_small_path(const ddq_ctx* c, char* why, int32_t cap) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (why && cap > 0) snprintf(why, (size_t)cap, "%s", c->small_off.c_str());
  return c->nb.small ? 1 : 0;
}

// ---------------- parameters ----------------
int64_t ddq_num_params(const ddq_ctx* c) { return c ? c->nb.L.total : -1; }

int ddq_param_layout(const ddq_ctx* c, ddq_blob_desc* out, int32_t cap, int32_t* n) {
  if (!c || !n) return fail(nullptr, DDQ_EINVAL, "null argument");
  const ParamLayout& L = c->nb.L;
  const char* names[5] = {"Qconv1", "Qconv2", "Qconv3", "Qfc4", "Q_out"};
  const int cout[3] = {32, 64, 64}, cin[3] = {4, 32, 64}, ks[3] = {7, 5, 3};
  *n = 10;
  if (!out) return DDQ_OK;
  if (cap < 10) return fail(const_cast<ddq_ctx*>(c), DDQ_EINVAL, "layout needs 10 entries");
  for (int l = 0; l < 5; ++l) {
    for (int i = 0; i < 2; ++i) {
      ddq_blob_desc& d = out[2 * l + i];
      memset(&d, 0, sizeof(d));
      snprintf(d.name, sizeof(d.name), "%s", names[l]);
      d.index = i;
      if (i == 0) {
        if (l < 3) { d.shape[0] = cout[l]; d.shape[1] = cin[l]; d.shape[2] = ks[l]; d.shape[3] = ks[l]; }
        else { d.shape[0] = 1; d.shape[1] = 1; d.shape[2] = l == 3 ? 512 : 4;
               d.shape[3] = l == 3 ? (int)(64 * L.S4 * L.S4) : 512; }
        d.offset = L.w[l]; d.count = L.wn[l];
      } else {
        d.shape[0] = 1; d.shape[1] = 1; d.shape[2] = 1; d.shape[3] = (int)L.bn[l];
        d.offset = L.b[l]; d.count = L.bn[l];
      }
    }
  }
  return DDQ_OK;
}

static int copy_in(ddq_ctx* c, float* dst, const float* src, int64_t n, int on_dev) {
  HIP_TRY(c, hipMemcpyAsync(dst, src, n * sizeof(float),
                            on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
  return DDQ_OK;
}
static int copy_out(ddq_ctx* c, float* dst, const float* src, int64_t n, int on_dev) {
  HIP_TRY(c, hipMemcpyAsync(dst, src, n * sizeof(float),
                            on_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_set_params(ddq_ctx* c, int32_t which, const float* src, int64_t n, int32_t on_dev) {
  if (!c || !src) return fail(c, DDQ_EINVAL, "null argument");
  if (which != 0 && which != 1) return fail(c, DDQ_EINVAL, "which must be 0 (Q) or 1 (P)");
  if (n != c->nb.L.total)
    return fail(c, DDQ_EINVAL, "expected %lld params, got %lld", (long long)c->nb.L.total, (long long)n);
  TRY(set_dev(c));
  TRY(copy_in(c, c->nb.theta[which], src, n, on_dev));
  HIP_TRY(c, launch_relayout(c->nb, which, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_get_params(ddq_ctx* c, int32_t which, float* dst, int64_t n, int32_t on_dev) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (which != 0 && which != 1) return fail(c, DDQ_EINVAL, "which must be 0 (Q) or 1 (P)");
  if (n != c->nb.L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  TRY(set_dev(c));
  return copy_out(c, dst, c->nb.theta[which], n, on_dev);
}

int ddq_get_grads(ddq_ctx* c, float* dst, int64_t n, int32_t on_dev) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (n != c->nb.L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  TRY(set_dev(c));
  return copy_out(c, dst, c->nb.grad, n, on_dev);
}

int ddq_set_grads(ddq_ctx* c, const float* src, int64_t n, int32_t on_dev) {
  if (!c || !src) return fail(c, DDQ_EINVAL, "null argument");
  if (n != c->nb.L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  TRY(set_dev(c));
  TRY(copy_in(c, c->nb.grad, src, n, on_dev));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_sync_target(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  HIP_TRY(c, hipMemcpyAsync(c->nb.theta[1], c->nb.theta[0], c->nb.L.total * 4,
                            hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->nb.wks[1], c->nb.wks[0], c->nb.L.wks_total * 3 * 2,
                            hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

// ---------------- replay ----------------
static int push_meta(ddq_ctx* c) {
  int64_t hv[2] = {c->head, c->valid};
  HIP_TRY(c, hipMemcpyAsync(c->r_meta, hv, sizeof(hv), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_replay_create(ddq_ctx* c, int64_t capacity) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (capacity < 2 || capacity > (int64_t)INT32_MAX)
    return fail(c, DDQ_EINVAL, "capacity must be in [2, 2^31) (got %lld)", (long long)capacity);
  if (c->r_state) return fail(c, DDQ_ESTATE, "replay already created");
  TRY(set_dev(c));
  const size_t slot = (size_t)4 * c->nb.S * c->nb.S;
  TRY(dalloc(c, &c->r_state, slot * capacity));
  TRY(dalloc(c, &c->r_action, (size_t)capacity));
  TRY(dalloc(c, &c->r_reward, (size_t)capacity));
  TRY(dalloc(c, &c->r_nonterm, (size_t)capacity));
  c->capacity = capacity;
  c->head = c->valid = 0;
  ReplayMeta m{};
  m.capacity = capacity;
  HIP_TRY(c, scopy(c, c->r_meta, &m, sizeof(m), hipMemcpyHostToDevice));
  invalidate_graph(c);
  return DDQ_OK;
}

int ddq_replay_add(ddq_ctx* c, int32_t action, int32_t reward, const uint8_t* state) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer (call ddq_replay_create)");
  if (action < 0 || action > 255) return fail(c, DDQ_EINVAL, "action must fit uint8");
  if (reward < -32768 || reward > 32767) return fail(c, DDQ_EINVAL, "reward must fit int16");
  TRY(set_dev(c));
  const size_t slot = (size_t)4 * c->nb.S * c->nb.S;
  const int64_t h = c->head;
  uint8_t a = (uint8_t)action, nt = state ? 1 : 0;
  int16_t r = (int16_t)reward;
  HIP_TRY(c, hipMemcpyAsync(c->r_action + h, &a, 1, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->r_reward + h, &r, 2, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->r_nonterm + h, &nt, 1, hipMemcpyHostToDevice, c->stream));
  if (state)
    HIP_TRY(c, hipMemcpyAsync(c->r_state + h * slot, state, slot, hipMemcpyHostToDevice, c->stream));
  c->head = (c->head + 1) % c->capacity;
  c->valid = std::min(c->capacity, c->valid + 1);
  return push_meta(c);
}

int ddq_replay_info(const ddq_ctx* c, int64_t* head, int64_t* valid, int64_t* capacity) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (head) *head = c->head;
  if (valid) *valid = c->valid;
  if (capacity) *capacity = c->capacity;
  return DDQ_OK;
}

int ddq_replay_import(ddq_ctx* c, const uint8_t* state, const uint8_t* action,
                      const int16_t* reward, const uint8_t* nonterm, int64_t n, int64_t head,
                      int64_t valid) {
  if (!c || !state || !action || !reward || !nonterm) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (n != c->capacity) return fail(c, DDQ_EINVAL, "import size %lld != capacity %lld",
                                    (long long)n, (long long)c->capacity);
  if (head < 0 || head >= n || valid < 0 || valid > n)
    return fail(c, DDQ_EINVAL, "head/valid out of range");
  TRY(set_dev(c));
  const size_t slot = (size_t)4 * c->nb.S * c->nb.S;
  HIP_TRY(c, scopy(c, c->r_state, state, slot * n, hipMemcpyHostToDevice));
  HIP_TRY(c, scopy(c, c->r_action, action, n, hipMemcpyHostToDevice));
  HIP_TRY(c, scopy(c, c->r_reward, reward, 2 * n, hipMemcpyHostToDevice));
  HIP_TRY(c, scopy(c, c->r_nonterm, nonterm, n, hipMemcpyHostToDevice));
  c->head = head;
  c->valid = valid;
  return push_meta(c);
}

int ddq_replay_export(ddq_ctx* c, uint8_t* state, uint8_t* action, int16_t* reward,
                      uint8_t* nonterm, int64_t n) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (n != c->capacity) return fail(c, DDQ_EINVAL, "export size mismatch");
  TRY(set_dev(c));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const size_t slot = (size_t)4 * c->nb.S * c->nb.S;
  if (state) HIP_TRY(c, scopy(c, state, c->r_state, slot * n, hipMemcpyDeviceToHost));
  if (action) HIP_TRY(c, scopy(c, action, c->r_action, n, hipMemcpyDeviceToHost));
  if (reward) HIP_TRY(c, scopy(c, reward, c->r_reward, 2 * n, hipMemcpyDeviceToHost));
  if (nonterm) HIP_TRY(c, scopy(c, nonterm, c->r_nonterm, n, hipMemcpyDeviceToHost));
  return DDQ_OK;
}

static int check_err_flag(ddq_ctx* c) {
  ReplayMeta m;
  HIP_TRY(c, hipMemcpyAsync(&m, c->r_meta, sizeof(m), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (m.err) {
    int32_t z = 0;
    HIP_TRY(c, scopy(c, reinterpret_cast<char*>(c->r_meta) + offsetof(ReplayMeta, err), &z, 4,
                         hipMemcpyHostToDevice));
    if (m.err == 2) return fail(c, DDQ_ERANGE, "batch sampler could not find distinct indices");
    return fail(c, DDQ_ERANGE, "stored action index out of range for %d actions", 4);
  }
  return DDQ_OK;
}

int ddq_replay_sample(ddq_ctx* c, const int32_t* idx, int32_t batch) {
  if (!c || !idx) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (batch >= c->valid)
    return fail(c, DDQ_EINVAL, "Can't draw sample of size %d from replay dataset of size %lld",
                batch, (long long)c->valid);
  if (batch != c->nb.B)
    return fail(c, DDQ_EINVAL, "sample size %d != net batch %d", batch, c->nb.B);
  for (int i = 0; i < batch; ++i) {
    if (idx[i] < 0 || idx[i] >= c->valid) return fail(c, DDQ_EINVAL, "index %d out of [0,valid)", idx[i]);
    if (i && idx[i] <= idx[i - 1]) return fail(c, DDQ_EINVAL, "indices must be sorted and distinct");
  }
  TRY(set_dev(c));
  HIP_TRY(c, hipMemcpyAsync(c->nb.idx, idx, batch * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_gather(c->nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                           c->stream));
  return check_err_flag(c);
}

int ddq_replay_sample_device_async(ddq_ctx* c, uint64_t seed) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (c->nb.B >= c->valid)
    return fail(c, DDQ_EINVAL, "Can't draw sample of size %d from replay dataset of size %lld",
                c->nb.B, (long long)c->valid);
  TRY(set_dev(c));
  HIP_TRY(c, launch_sample(c->nb, c->r_meta, seed, c->stream));
  HIP_TRY(c, launch_gather(c->nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                           c->stream));
  return DDQ_OK;
}

int ddq_replay_fill_tiled(ddq_ctx* c, const uint8_t* state, const uint8_t* action,
                          const int16_t* reward, const uint8_t* nonterm, int64_t pool,
                          int64_t head, int64_t valid) {
  if (!c || !state || !action || !reward || !nonterm) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  const int64_t n = c->capacity;
  if (pool < 1 || pool > n) return fail(c, DDQ_EINVAL, "pool must be in [1, capacity]");
  if (head < 0 || head >= n || valid < 0 || valid > n)
    return fail(c, DDQ_EINVAL, "head/valid out of range");
  TRY(set_dev(c));
  const size_t slot = (size_t)4 * c->nb.S * c->nb.S;
  HIP_TRY(c, scopy(c, c->r_state, state, slot * pool, hipMemcpyHostToDevice));
  if (pool < n)
    HIP_TRY(c, launch_tile(c->r_state + slot * pool, c->r_state, slot * pool,
                           slot * (n - pool), c->stream));
  std::vector<uint8_t> a(n), t(n);
  std::vector<int16_t> r(n);
  for (int64_t i = 0; i < n; ++i) {
    a[i] = action[i % pool]; r[i] = reward[i % pool]; t[i] = nonterm[i % pool];
  }
  HIP_TRY(c, scopy(c, c->r_action, a.data(), n, hipMemcpyHostToDevice));
  HIP_TRY(c, scopy(c, c->r_reward, r.data(), 2 * n, hipMemcpyHostToDevice));
  HIP_TRY(c, scopy(c, c->r_nonterm, t.data(), n, hipMemcpyHostToDevice));
  c->head = head;
  c->valid = valid;
  return push_meta(c);
}

static int check_batch_out(ddq_ctx* c, int32_t n, float* s0, float* a, float* r, float* s1,
                           float* nt) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!s0 || !a || !r || !s1 || !nt) return fail(c, DDQ_EINVAL, "null output buffer");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (n < 1) return fail(c, DDQ_EINVAL, "n must be >= 1");
  if ((int64_t)n * c->nb.S * c->nb.S >= (int64_t)1 << 31)
    return fail(c, DDQ_EINVAL, "n * S^2 must be < 2^31 (n=%d)", n);
  if (n >= c->valid)
    return fail(c, DDQ_EINVAL, "Can't draw sample of size %d from replay dataset of size %lld",
                n, (long long)c->valid);
  return DDQ_OK;
}

int ddq_replay_sample_batch_async(ddq_ctx* c, int32_t n, uint64_t seed, int32_t* idx,
                                  float* state, float* action, float* reward, float* next_state,
                                  float* nonterm) {
  TRY(check_batch_out(c, n, state, action, reward, next_state, nonterm));
  if (!idx) return fail(c, DDQ_EINVAL, "null idx");
  if (2 * (int64_t)n > c->valid)
    return fail(c, DDQ_EINVAL, "batch sampler needs n <= valid/2 (n=%d, valid=%lld)", n,
                (long long)c->valid);
  TRY(set_dev(c));
  if (!c->r_bitmap) {   // sized for the full ring: valid never exceeds capacity
    const int64_t nblk = ((c->capacity + 31) / 32 + 1023) / 1024;
    TRY(dalloc(c, &c->r_bitmap, (size_t)nblk * 1024));
    TRY(dalloc(c, &c->r_blk, (size_t)nblk));
  }
  HIP_TRY(c, launch_sample_batch(c->r_meta, c->valid, n, seed, c->batch_ctr++, c->r_bitmap,
                                 c->r_blk, idx, c->stream));
  HIP_TRY(c, launch_gather_nchw(c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                                idx, n, c->nb.S, state, next_state, action, reward, nonterm,
                                c->stream));
  return DDQ_OK;
}

int ddq_replay_gather_batch_async(ddq_ctx* c, const int32_t* idx, int32_t n, float* state,
                                  float* action, float* reward, float* next_state,
                                  float* nonterm) {
  TRY(check_batch_out(c, n, state, action, reward, next_state, nonterm));
  if (!idx) return fail(c, DDQ_EINVAL, "null idx");
  TRY(set_dev(c));
  HIP_TRY(c, launch_gather_nchw(c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                                idx, n, c->nb.S, state, next_state, action, reward, nonterm,
                                c->stream));
  return DDQ_OK;
}

int ddq_index_log_enable(ddq_ctx* c, int64_t draws) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (draws < 0 || draws > (1ll << 24)) return fail(c, DDQ_EINVAL, "draws must be in [0, 2^24]");
  TRY(set_dev(c));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // the ring restarts at the current draw: earlier draws (or entries of a
  // ring of another capacity) are never reported as logged
  ReplayMeta m;
  HIP_TRY(c, scopy(c, &m, c->r_meta, sizeof(m), hipMemcpyDeviceToHost));
  c->log_first = (int64_t)m.counter;
  if (draws == 0) {
    c->nb.idx_log = nullptr;
    c->nb.log_cap = 0;
  } else if (draws > c->log_buf_cap) {
    TRY(dalloc(c, &c->log_buf, (size_t)draws * c->nb.B));
    c->log_buf_cap = draws;
    c->nb.idx_log = c->log_buf;
    c->nb.log_cap = draws;
  } else {
    c->nb.idx_log = c->log_buf;
    c->nb.log_cap = draws;
  }
  invalidate_graph(c);   // captured kernels hold the log pointer
  return DDQ_OK;
}

int ddq_replay_draws(ddq_ctx* c, int64_t* draws) {
  if (!c || !draws) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  TRY(set_dev(c));
  ReplayMeta m;
  HIP_TRY(c, hipMemcpyAsync(&m, c->r_meta, sizeof(m), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  *draws = (int64_t)m.counter;
  return DDQ_OK;
}

int ddq_index_log_read(ddq_ctx* c, int64_t first, int64_t n, int32_t* out) {
  if (!c || !out) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->nb.idx_log) return fail(c, DDQ_ESTATE, "index log not enabled");
  int64_t drawn = 0;
  TRY(ddq_replay_draws(c, &drawn));
  if (first < c->log_first || n < 0 || first + n > drawn || drawn - first > c->nb.log_cap)
    return fail(c, DDQ_EINVAL,
                "draws [%lld, %lld) not in the log (logged from draw %lld, drawn %lld, cap %lld)",
                (long long)first, (long long)(first + n), (long long)c->log_first,
                (long long)drawn, (long long)c->nb.log_cap);
  const int B = c->nb.B;
  for (int64_t d = first; d < first + n; ++d)
    HIP_TRY(c, hipMemcpyAsync(out + (d - first) * B, c->nb.idx_log + (d % c->nb.log_cap) * B,
                              (size_t)B * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_replay_status(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  TRY(set_dev(c));
  return check_err_flag(c);
}

int ddq_read_indices(ddq_ctx* c, int32_t* idx, int32_t batch) {
  if (!c || !idx || batch != c->nb.B) return fail(c, DDQ_EINVAL, "bad argument");
  TRY(set_dev(c));
  HIP_TRY(c, hipMemcpyAsync(idx, c->nb.idx, batch * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_read_minibatch(ddq_ctx* c, float* state, float* action, float* reward, float* next_state,
                       float* nonterm) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  const int B = c->nb.B, SS = c->nb.S * c->nb.S;
  std::vector<float> tmp((size_t)B * SS * 4);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int which = 0; which < 2; ++which) {
    float* dst = which ? next_state : state;
    if (!dst) continue;
    HIP_TRY(c, scopy(c, tmp.data(), which ? c->nb.next_state : c->nb.state, tmp.size() * 4,
                         hipMemcpyDeviceToHost));
    for (int b = 0; b < B; ++b)
      for (int ch = 0; ch < 4; ++ch)
        for (int p = 0; p < SS; ++p)
          dst[((size_t)b * 4 + ch) * SS + p] = tmp[((size_t)b * SS + p) * 4 + ch];
  }
  if (action) HIP_TRY(c, scopy(c, action, c->nb.action, B * 16, hipMemcpyDeviceToHost));
  if (reward) HIP_TRY(c, scopy(c, reward, c->nb.reward, B * 4, hipMemcpyDeviceToHost));
  if (nonterm) HIP_TRY(c, scopy(c, nonterm, c->nb.nonterm, B * 4, hipMemcpyDeviceToHost));
  return DDQ_OK;
}

int ddq_write_minibatch(ddq_ctx* c, const float* state, const float* action, const float* reward,
                        const float* next_state, const float* nonterm) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  const int B = c->nb.B, SS = c->nb.S * c->nb.S;
  std::vector<float> tmp((size_t)B * SS * 4);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int which = 0; which < 2; ++which) {
    const float* src = which ? next_state : state;
    if (!src) continue;
    for (int b = 0; b < B; ++b)
      for (int ch = 0; ch < 4; ++ch)
        for (int p = 0; p < SS; ++p)
          tmp[((size_t)b * SS + p) * 4 + ch] = src[((size_t)b * 4 + ch) * SS + p];
    HIP_TRY(c, scopy(c, which ? c->nb.next_state : c->nb.state, tmp.data(), tmp.size() * 4,
                         hipMemcpyHostToDevice));
  }
  if (action) HIP_TRY(c, scopy(c, c->nb.action, action, B * 16, hipMemcpyHostToDevice));
  if (reward) HIP_TRY(c, scopy(c, c->nb.reward, reward, B * 4, hipMemcpyHostToDevice));
  if (nonterm) HIP_TRY(c, scopy(c, c->nb.nonterm, nonterm, B * 4, hipMemcpyHostToDevice));
  return DDQ_OK;
}

// ---------------- compute ----------------
// book >= 0: this backward feeds a step's apply; its slab reduce also does
// the apply bookkeeping with target period `book` (saves a launch).
static int enqueue_fwd_bwd(ddq_ctx* c, const NetBuffers& nb, void (*mark)(void*, const char*),
                           void* marg, int book = -1, ReplayMeta* bump = nullptr) {
  if (nb.small) {
    HIP_TRY(c, launch_small_fwd_head(nb, c->stream, mark, marg));
  } else {
    HIP_TRY(c, launch_forward(nb, 2, c->stream, mark, marg, false));
    if (mark) mark(marg, "head");
    HIP_TRY(c, launch_head(nb, c->stream));
  }
  // one stream: forking the weight-gradient kernels onto a side stream cost
  // more in cross-stream graph edges (6-14 us idle each, measured) than the
  // overlap returned, as every kernel here fills the GPU on its own
  if (nb.small)
    HIP_TRY(c, launch_small_bwd(nb, c->stream, mark, marg, book >= 0, book, bump, nullptr, nullptr,
                                nullptr));
  else
    HIP_TRY(c, launch_backward(nb, c->stream, mark, marg, book >= 0, book, bump));
  return DDQ_OK;
}
static int enqueue_fwd_bwd(ddq_ctx* c, void (*mark)(void*, const char*), void* marg) {
  return enqueue_fwd_bwd(c, c->nb, mark, marg);
}

int ddq_forward_backward_async(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  return enqueue_fwd_bwd(c, nullptr, nullptr);
}

int ddq_forward_backward(ddq_ctx* c, float* loss) {
  TRY(ddq_forward_backward_async(c));
  if (loss) return copy_out(c, loss, c->nb.loss, 1, 0);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_forward_q(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  HIP_TRY(c, launch_act(c->nb, c->nb.state, c->nb.B, c->act_p3, c->act_h4, c->act_part,
                        c->nb.q_out, nullptr, c->act_p1s, c->act_p2s, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_read_blob(ddq_ctx* c, const char* name, float* dst, int64_t n) {
  if (!c || !name || !dst) return fail(c, DDQ_EINVAL, "null argument");
  const int B = c->nb.B;
  struct { const char* nm; float* p; int64_t cnt; } t[] = {
      {"Q_out", c->nb.q_out, 4ll * B}, {"P_out", c->nb.p_out, 4ll * B},
      {"Q_sa", c->nb.q_sa, B},         {"P_sa", c->nb.p_sa, B},
      {"target_Q_sa", c->nb.target, B}, {"loss", c->nb.loss, 1}};
  for (auto& e : t) {
    if (strcmp(e.nm, name) == 0) {
      if (n != e.cnt) return fail(c, DDQ_EINVAL, "blob %s has %lld elements", name, (long long)e.cnt);
      TRY(set_dev(c));
      return copy_out(c, dst, e.p, n, 0);
    }
  }
  return fail(c, DDQ_EINVAL, "unknown blob '%s'", name);
}

int ddq_read_pool_mask(ddq_ctx* c, int32_t layer, uint8_t* dst, int64_t n) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (layer < 1 || layer > 3) return fail(c, DDQ_EINVAL, "layer must be 1..3");
  const int B = c->nb.B, C = layer == 1 ? 32 : 64, Hp = c->nb.S >> layer;
  const int64_t cnt = (int64_t)B * C * Hp * Hp;
  if (n != cnt) return fail(c, DDQ_EINVAL, "mask %d has %lld elements", layer, (long long)cnt);
  TRY(set_dev(c));
  std::vector<uint8_t> tmp(cnt);
  const uint8_t* src = layer == 1 ? c->nb.mask1 : (layer == 2 ? c->nb.mask2 : c->nb.mask3);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  HIP_TRY(c, scopy(c, tmp.data(), src, cnt, hipMemcpyDeviceToHost));
  for (int b = 0; b < B; ++b)
    for (int ch = 0; ch < C; ++ch)
      for (int p = 0; p < Hp * Hp; ++p)
        dst[((size_t)b * C + ch) * Hp * Hp + p] = tmp[((size_t)b * Hp * Hp + p) * C + ch];
  return DDQ_OK;
}

int ddq_select_action(ddq_ctx* c, const uint8_t* states, int32_t n, int32_t* actions) {
  if (!c || !states || !actions) return fail(c, DDQ_EINVAL, "null argument");
  if (n < 1 || n > c->nb.B) return fail(c, DDQ_EINVAL, "n must be in [1,B]");
  TRY(set_dev(c));
  const size_t bytes = (size_t)n * 4 * c->nb.S * c->nb.S;
  HIP_TRY(c, hipMemcpyAsync(c->act_u8, states, bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, launch_u8_to_nhwc(c->act_u8, n, c->nb.S, c->act_in, c->stream));
  HIP_TRY(c, launch_act(c->nb, c->act_in, n, c->act_p3, c->act_h4, c->act_part, c->act_q,
                        c->act_out, c->act_p1s, c->act_p2s, c->stream));
  HIP_TRY(c, hipMemcpyAsync(actions, c->act_out, n * 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

// ---------------- apply ----------------
static int check_cfg(ddq_ctx* c, const ddq_update_cfg* u) {
  if (!u) return fail(c, DDQ_EINVAL, "null update cfg");
  if (u->rule < 0 || u->rule > 3) return fail(c, DDQ_EINVAL, "unknown update rule %d", u->rule);
  return DDQ_OK;
}

int ddq_apply_async(ddq_ctx* c, const ddq_update_cfg* u) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(check_cfg(c, u));
  TRY(set_dev(c));
  HIP_TRY(c, launch_apply(c->nb, u->rule, u->lr, u->decay, u->eps, u->momentum, u->weight_decay,
                          0, false, c->stream));
  c->applied++;
  return DDQ_OK;
}

int ddq_apply(ddq_ctx* c, const ddq_update_cfg* u) {
  TRY(ddq_apply_async(c, u));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_reset_optimizer(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  TRY(set_dev(c));
  HIP_TRY(c, hipMemsetAsync(c->nb.opt, 0, c->nb.L.total * 4, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->nb.opt_init, 0, 4, c->stream));
  HIP_TRY(c, hipMemsetAsync(c->nb.iter, 0, 8, c->stream));
  c->applied = 0;
  c->steps = 0;
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

int ddq_get_optimizer_state(ddq_ctx* c, float* dst, int64_t n) {
  if (!c || !dst) return fail(c, DDQ_EINVAL, "null argument");
  if (n != c->nb.L.total) return fail(c, DDQ_EINVAL, "size mismatch");
  TRY(set_dev(c));
  return copy_out(c, dst, c->nb.opt, n, 0);
}

// ---------------- comm ----------------
int ddq_comm_get_unique_id(uint8_t id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "unique id size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(nullptr, DDQ_ERCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  memcpy(id, &u, 128);
  return DDQ_OK;
}

// Shard geometry and exchange buffers for W ranks (RCCL or in-process).
static int setup_shards(ddq_ctx* c, int W) {
  const int64_t P = c->nb.L.total;
  c->shard_len = ((P + (int64_t)W * 64 - 1) / ((int64_t)W * 64)) * 64;
  if (!c->cs) {
    HIP_TRY(c, hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
    for (auto& e : c->cev) HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // exchange buffers are allocated once for the largest W (kMaxRanks slices
  // of at most P/W + 64 floats fit in P + kShardPad ... per slice set)
  if (!c->gsl) TRY(dalloc(c, &c->gsl, (size_t)P + kShardPad));
  return DDQ_OK;
}

int ddq_comm_init(ddq_ctx* c, const uint8_t id[128], int32_t nranks, int32_t rank) {
  if (!c || !id) return fail(c, DDQ_EINVAL, "null argument");
  if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
    return fail(c, DDQ_EINVAL, "bad rank/nranks (nranks <= %d)", kMaxRanks);
  if (c->local) return fail(c, DDQ_ESTATE, "ctx belongs to an in-process group");
  TRY(set_dev(c));
  if (c->comm) ncclCommDestroy(c->comm);
  c->comm = nullptr;
  ncclUniqueId u;
  memcpy(&u, id, 128);
  NCCL_TRY(c, ncclCommInitRank(&c->comm, nranks, u, rank));
  c->nranks = nranks;
  c->rank = rank;
  TRY(setup_shards(c, nranks));
  invalidate_graph(c);
  return DDQ_OK;
}

int ddq_allreduce_grads_async(ddq_ctx* c) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!c->comm) return fail(c, DDQ_ESTATE, "no communicator (call ddq_comm_init)");
  TRY(set_dev(c));
  NCCL_TRY(c, ncclAllReduce(c->nb.grad, c->nb.grad, (size_t)c->nb.L.total, ncclFloat, ncclSum,
                            c->comm, c->stream));
  return DDQ_OK;
}

int ddq_allreduce_grads(ddq_ctx* c) {
  TRY(ddq_allreduce_grads_async(c));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return DDQ_OK;
}

// ---------------- step ----------------
static bool has_exchange(const ddq_ctx* c, const ddq_step_cfg* cfg) {
  return cfg->exchange != DDQ_EXCHANGE_NONE && (c->comm != nullptr || c->local);
}
// param-server iterations one step consumes (server.py:200 INCR per gradient)
static int step_inc(const ddq_ctx* c, const ddq_step_cfg* cfg) {
  return (has_exchange(c, cfg) &&
          (cfg->exchange == DDQ_EXCHANGE_SERVER || cfg->exchange == DDQ_EXCHANGE_ASYNC))
             ? c->nranks
             : 1;
}
static bool is_async(const ddq_ctx* c, const ddq_step_cfg* cfg) {
  return has_exchange(c, cfg) && cfg->exchange == DDQ_EXCHANGE_ASYNC;
}
// Once the async exchange began, the central model lives in the owners'
// shards: other step kinds would train a replica the owners never see.
static int check_not_async(ddq_ctx* c) {
  if (c->async_on)
    return fail(c, DDQ_ESTATE, "the async exchange is in progress on this ctx (its central "
                               "model lives in the owners' shards): async steps only");
  return DDQ_OK;
}

// Overlapped all-reduce, part 1 (called by launch_backward right after the
// fc4 weight-gradient kernel): the comm stream sums the fc4 weight bucket
// (2.1 M of the 2.2 M parameters at 64x64) while the conv backward runs;
// cev[2] marks it done (the fused apply's slab-reduce launch waits for it).
static hipError_t fc4_bucket_start(void* arg) {
  ddq_ctx* c = reinterpret_cast<ddq_ctx*>(arg);
  const ParamLayout& L = c->nb.L;
  hipError_t e = hipEventRecord(c->cev[0], c->stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->cs, c->cev[0], 0);
  if (e != hipSuccess) return e;
  ncclResult_t r = ncclAllReduce(c->nb.grad + L.w[3], c->nb.grad + L.w[3], (size_t)L.wn[3],
                                 ncclFloat, ncclSum, c->comm, c->cs);
  if (r != ncclSuccess) {
    c->comm_err = ncclGetErrorString(r);
    return hipErrorUnknown;
  }
  return hipEventRecord(c->cev[2], c->cs);
}

static int enqueue_fwd_bwd_x(ddq_ctx* c, const NetBuffers& nb, void (*mark)(void*, const char*),
                             void* marg, int book, ReplayMeta* bump, bool overlap,
                             const Prefetch* pf = nullptr) {
  if (nb.small) {
    HIP_TRY(c, launch_small_fwd_head(nb, c->stream, mark, marg, bump, nb.fa.on ? pf : nullptr));
  } else {
    HIP_TRY(c, launch_forward(nb, 2, c->stream, mark, marg, false));
    if (mark) mark(marg, "head");
    // fused apply: the draw counter advances here (pipelined: with the next
    // step's draw, kernels.hip head_draw)
    HIP_TRY(c, launch_head(nb, c->stream, bump, nb.fa.on ? pf : nullptr));
  }
  hipError_t e = nb.small ? launch_small_bwd(nb, c->stream, mark, marg, book >= 0, book, bump,
                                             overlap ? fc4_bucket_start : nullptr, c, pf)
                          : launch_backward(nb, c->stream, mark, marg, book >= 0, book, bump,
                                            overlap ? fc4_bucket_start : nullptr, c, pf);
  if (e != hipSuccess && !c->comm_err.empty()) {
    std::string m = c->comm_err;
    c->comm_err.clear();
    return fail(c, DDQ_ERCCL, "overlapped all-reduce: %s", m.c_str());
  }
  HIP_TRY(c, e);
  return DDQ_OK;
}

// Gradient exchange + apply of one step over RCCL (graph-capturable):
//  ALLREDUCE  sum all-reduce, replicated apply (overlap: fc4 bucket on the
//             comm stream under the conv backward, applied by the slab-reduce
//             launch (nb.fa.ext); the rest -- conv layers, fc4 bias, Q_out --
//             as one grouped call after the slab reduce, then their apply);
//  SHARDED    reduce-scatter(sum) -> owner apply of its 1/W shard ->
//             in-place all-gather of theta -> conv layouts / P <- Q refresh;
//  SERVER     all-to-all of gradient slices -> owner applies the W gradients
//             one by one in rank order (server.py:196-209 on arrival) ->
//             all-gather -> refresh.
static int enqueue_exchange_apply(ddq_ctx* c, const ddq_step_cfg* cfg, const NetBuffers& nb,
                                  void (*mark)(void*, const char*), void* marg, bool overlap,
                                  const Prefetch* pf = nullptr) {
  const ddq_update_cfg& u = cfg->update;
  const ParamLayout& L = nb.L;
  const int ex = has_exchange(c, cfg) ? cfg->exchange : DDQ_EXCHANGE_NONE;
  if (ex == DDQ_EXCHANGE_NONE || ex == DDQ_EXCHANGE_ALLREDUCE) {
    if (ex == DDQ_EXCHANGE_ALLREDUCE) {
      if (mark) mark(marg, "allreduce");
      if (overlap && nb.fa.on) {
        // fc4's weights were summed under the conv backward and applied by
        // the slab-reduce launch (nb.fa.ext), whose stream waited for that
        // all-reduce: the rest (4 % of the parameters) right here on the ctx
        // stream -- nothing is left to overlap it with, and a comm-stream
        // round trip costs a graph fork / join (measured 0.968 against 0.995
        // of the exchange-free step at world 1 with it)
        NCCL_TRY(c, ncclGroupStart());
        NCCL_TRY(c, ncclAllReduce(nb.grad, nb.grad, (size_t)L.w[3], ncclFloat, ncclSum, c->comm,
                                  c->stream));
        NCCL_TRY(c, ncclAllReduce(nb.grad + L.b[3], nb.grad + L.b[3], (size_t)(L.total - L.b[3]),
                                  ncclFloat, ncclSum, c->comm, c->stream));
        NCCL_TRY(c, ncclGroupEnd());
      } else if (overlap) {
        HIP_TRY(c, hipEventRecord(c->cev[0], c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->cs, c->cev[0], 0));
        NCCL_TRY(c, ncclGroupStart());
        NCCL_TRY(c, ncclAllReduce(nb.grad, nb.grad, (size_t)L.w[3], ncclFloat, ncclSum, c->comm,
                                  c->cs));
        NCCL_TRY(c, ncclAllReduce(nb.grad + L.b[3], nb.grad + L.b[3], (size_t)(L.total - L.b[3]),
                                  ncclFloat, ncclSum, c->comm, c->cs));
        NCCL_TRY(c, ncclGroupEnd());
        HIP_TRY(c, hipEventRecord(c->cev[1], c->cs));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->cev[1], 0));
      } else {
        NCCL_TRY(c, ncclAllReduce(nb.grad, nb.grad, (size_t)L.total, ncclFloat, ncclSum, c->comm,
                                  c->stream));
      }
    }
    if (mark) mark(marg, "apply");
    HIP_TRY(c, launch_apply(nb, u.rule, u.lr, u.decay, u.eps, u.momentum, u.weight_decay,
                            cfg->target_period, true, c->stream, pf));
    return DDQ_OK;
  }
  const int W = c->nranks;
  const size_t len = (size_t)c->shard_len;
  if (mark) mark(marg, ex == DDQ_EXCHANGE_SHARDED ? "reduce_scatter" : "all_to_all");
  if (ex == DDQ_EXCHANGE_SHARDED)
    NCCL_TRY(c, ncclReduceScatter(nb.grad, c->gsl, len, ncclFloat, ncclSum, c->comm, c->stream));
  else if (W > 1) {
    // all-to-all without the rank's own slice: the owner apply reads that one
    // in place from nb.grad (no self copy of len floats through RCCL)
    NCCL_TRY(c, ncclGroupStart());
    for (int p = 0; p < W; ++p) {
      if (p == c->rank) continue;
      NCCL_TRY(c, ncclSend(nb.grad + (size_t)p * len, len, ncclFloat, p, c->comm, c->stream));
      NCCL_TRY(c, ncclRecv(c->gsl + (size_t)p * len, len, ncclFloat, p, c->comm, c->stream));
    }
    NCCL_TRY(c, ncclGroupEnd());
  }
  if (mark) mark(marg, "apply_shard");
  HIP_TRY(c, launch_apply_shard(nb, u.rule, u.lr, u.decay, u.eps, u.momentum, u.weight_decay,
                                c->gsl, (int64_t)c->rank * len, (int64_t)len, (int64_t)len,
                                ex == DDQ_EXCHANGE_SHARDED ? 1 : W, c->stream, nullptr, -1, pf,
                                nullptr, -1, c->rank,
                                ex == DDQ_EXCHANGE_SHARDED ? nullptr
                                                           : nb.grad + (size_t)c->rank * len));
  if (mark) mark(marg, "all_gather");
  NCCL_TRY(c, ncclAllGather(nb.theta[0] + (size_t)c->rank * len, nb.theta[0], len, ncclFloat,
                            c->comm, c->stream));
  // the owner's shard was refreshed by its apply: the other ranks' shards
  // only (no launch when one rank owns every parameter)
  if (mark) mark(marg, "refresh");
  HIP_TRY(c, launch_refresh(nb, c->stream, -1, (int64_t)c->rank * len,
                            (int64_t)(c->rank + 1) * len));
  return DDQ_OK;
}

// fwd/bwd -> exchange -> apply on the minibatch held by `nb`; when `pre` is
// given, the NEXT step's sample + gather into `pre`'s minibatch set run on
// the side stream under this step's forward (the replay ring is not written
// inside a step, and the device RNG counter advances in the same order, so
// the index stream equals the sequential one).
// Pipelined steps whose next draw + gather ride on the apply launch (no side
// stream): exchanges that end in the plain apply kernel, B <= 256.
// (sharded / server: on the owner-apply launch, after the slab reduce's
// bookkeeping advanced the draw counter)
static bool fused_prefetch(const ddq_ctx* c, const ddq_step_cfg* cfg) {
  const int ex = has_exchange(c, cfg) ? cfg->exchange : DDQ_EXCHANGE_NONE;
  return ex != DDQ_EXCHANGE_ASYNC && c->nb.B <= 256;
}

static int enqueue_train(ddq_ctx* c, const ddq_step_cfg* cfg, const NetBuffers& nb_in,
                         const NetBuffers* pre, void (*mark)(void*, const char*), void* marg,
                         ReplayMeta* bump = nullptr) {
  NetBuffers nb = nb_in;
  nb.book_inc = step_inc(c, cfg);
  // exchange-free steps: fc4's weight update rides on the slab-reduce launch
  const int ex = has_exchange(c, cfg) ? cfg->exchange : DDQ_EXCHANGE_NONE;
  const bool ar_overlap = ex == DDQ_EXCHANGE_ALLREDUCE && cfg->overlap && c->comm;
  // (deepq16: fc4's parameters are final and applied inside the fc4 chain,
  // K2, before any bucket could be summed: the overlapped all-reduce takes the
  // plain apply launch there)
  if ((ex == DDQ_EXCHANGE_NONE || (ar_overlap && !nb.small)) && fused_apply_ok(nb.L)) {
    const ddq_update_cfg& u = cfg->update;
    nb.fa.on = 1;
    nb.fa.ext = ar_overlap ? 1 : 0;
    nb.fa.store_grad = ar_overlap || !(cfg->flags & DDQ_STEP_NO_GRAD_STORE);
    nb.fc4_wait = ar_overlap ? c->cev[2] : nullptr;
    nb.fa.rule = u.rule;
    nb.fa.period = cfg->target_period > 0 ? cfg->target_period : 0;
    nb.fa.lr = u.lr; nb.fa.decay = u.decay; nb.fa.eps = u.eps;
    nb.fa.momentum = u.momentum; nb.fa.wd = u.weight_decay;
  }
  if (pre && fused_prefetch(c, cfg)) {
    // the step's bookkeeping advances the draw counter (bump) before the apply
    // launch draws the next minibatch with it
    const Prefetch pf = make_prefetch(*pre, c->r_state, c->r_action, c->r_reward, c->r_nonterm,
                                      c->r_meta, cfg->seed);
    // fused apply: the slab-reduce launch carries the draw + gather too
    TRY(enqueue_fwd_bwd_x(c, nb, mark, marg, cfg->target_period > 0 ? cfg->target_period : 0,
                          c->r_meta, ar_overlap, nb.fa.on ? &pf : nullptr));
    return enqueue_exchange_apply(c, cfg, nb, mark, marg, ar_overlap, nb.fa.on ? nullptr : &pf);
  }
  if (pre) {
    HIP_TRY(c, hipEventRecord(nb.ev[6], c->stream));
    HIP_TRY(c, hipStreamWaitEvent(nb.side, nb.ev[6], 0));
    HIP_TRY(c, launch_sample(*pre, c->r_meta, cfg->seed, nb.side));
    HIP_TRY(c, launch_gather(*pre, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                             nb.side));
    HIP_TRY(c, hipEventRecord(nb.ev[7], nb.side));
  }
  TRY(enqueue_fwd_bwd_x(c, nb, mark, marg, cfg->target_period > 0 ? cfg->target_period : 0, bump,
                        ar_overlap));
  TRY(enqueue_exchange_apply(c, cfg, nb, mark, marg, ar_overlap));
  if (pre) HIP_TRY(c, hipStreamWaitEvent(c->stream, nb.ev[7], 0));
  return DDQ_OK;
}

static int enqueue_step(ddq_ctx* c, const ddq_step_cfg* cfg, void (*mark)(void*, const char*),
                        void* marg) {
  if (c->nb.B <= 256) {   // one kernel: every gather workgroup draws the same index set
    if (mark) mark(marg, "sample_gather");
    HIP_TRY(c, launch_sample_gather(c->nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm,
                                    c->r_meta, cfg->seed, c->stream));
    return enqueue_train(c, cfg, c->nb, nullptr, mark, marg, c->r_meta);
  }
  if (mark) mark(marg, "sample");
  HIP_TRY(c, launch_sample(c->nb, c->r_meta, cfg->seed, c->stream));
  if (mark) mark(marg, "gather");
  HIP_TRY(c, launch_gather(c->nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                           c->stream));
  return enqueue_train(c, cfg, c->nb, nullptr, mark, marg);
}

// minibatch set p: 0 = the ctx's own buffers, 1 = the pipelining twin
static NetBuffers mb_view(const ddq_ctx* c, int p) {
  NetBuffers v = c->nb;
  if (p == 1) {
    v.state = c->mb2_state; v.next_state = c->mb2_next; v.action = c->mb2_action;
    v.reward = c->mb2_reward; v.nonterm = c->mb2_nonterm; v.idx = c->mb2_idx;
  }
  return v;
}

// The pull at iteration 0 copies Q -> P (server.py:188-189, 0 % period == 0);
// later syncs are fused into the apply kernel of the preceding update.
static int initial_target_sync(ddq_ctx* c, const ddq_step_cfg* cfg) {
  if (cfg->target_period > 0 && c->applied % cfg->target_period == 0) {
    HIP_TRY(c, hipMemcpyAsync(c->nb.theta[1], c->nb.theta[0], c->nb.L.total * 4,
                              hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(c->nb.wks[1], c->nb.wks[0], c->nb.L.wks_total * 3 * 2,
                              hipMemcpyDeviceToDevice, c->stream));
  }
  return DDQ_OK;
}

static int check_step(ddq_ctx* c, const ddq_step_cfg* cfg) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (!cfg) return fail(c, DDQ_EINVAL, "null step cfg");
  TRY(check_cfg(c, &cfg->update));
  if (!c->r_state) return fail(c, DDQ_ESTATE, "no replay buffer");
  if (c->nb.B >= c->valid)
    return fail(c, DDQ_EINVAL, "Can't draw sample of size %d from replay dataset of size %lld",
                c->nb.B, (long long)c->valid);
  if (cfg->exchange < DDQ_EXCHANGE_NONE || cfg->exchange > DDQ_EXCHANGE_ASYNC)
    return fail(c, DDQ_EINVAL, "unknown exchange %d", cfg->exchange);
  if (cfg->flags & ~DDQ_STEP_NO_GRAD_STORE)
    return fail(c, DDQ_EINVAL, "unknown step flags 0x%x", (unsigned)cfg->flags);
  if (cfg->exchange != DDQ_EXCHANGE_NONE && c->nranks > 1 && !c->comm && !c->local)
    return fail(c, DDQ_ESTATE, "no communicator");
  return DDQ_OK;
}

// ---------------- asynchronous param server (DDQ_EXCHANGE_ASYNC) ----------------
// The reference's workers free-run (main.py:61-112: fetch -> experience ->
// full_pass -> push) against one server that applies every pushed gradient on
// arrival (server.py:196-209) and copies Q -> P on a pull that sees
// iteration % period == 0 (server.py:181-193).  Here rank r owns shard r of
// the central model and its optimizer state; a TICK is one push: worker w's
// gradient slices go to the owners, each owner applies its slice (iteration
// += 1), the owners send worker w their shards (and the central P's when a
// special update happened since w's last pull), and w computes its next
// gradient on the model it pulled while the other ticks proceed.  Which
// worker pushes at each tick is the arrival order: round-robin (the
// deterministic test schedule, one step = W ticks) or ticket order (the
// worker whose gradient is ready first; ddq_async_tick / ddq_group_async_run).

// Worker side: the minibatch draw + gather and the forward/backward on the
// model this worker last pulled (no apply bookkeeping: the owners keep the
// iteration), into nb.grad, on the ctx stream; grad_ev marks it ready.
// drawn: the minibatch was drawn + gathered already (by the owner apply of
// this worker's own push, async_owner_apply)
static int async_compute(ddq_ctx* c, const ddq_step_cfg* cfg, bool drawn = false) {
  NetBuffers nb = c->nb;
  if (nb.B <= 256) {   // one draw + gather launch; the head advances the counter
    nb.head_bump = 1;
    if (!drawn)
      HIP_TRY(c, launch_sample_gather(nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm,
                                      c->r_meta, cfg->seed, c->stream));
    TRY(enqueue_fwd_bwd_x(c, nb, nullptr, nullptr, -1, c->r_meta, false));
  } else {
    HIP_TRY(c, launch_sample(nb, c->r_meta, cfg->seed, c->stream));
    HIP_TRY(c, launch_gather(nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                             c->stream));
    TRY(enqueue_fwd_bwd_x(c, nb, nullptr, nullptr, -1, nullptr, false));
  }
  HIP_TRY(c, hipEventRecord(c->grad_ev, c->stream));
  c->ready_seen = false;
  c->grad_ev_captured = c->acapture;
  return DDQ_OK;
}

// The special update (server.py:186-189) runs when a pull sees iteration %
// period == 0; with one pull per tick that is every multiple of the period, so
// a worker's P must be re-pulled iff a multiple lies in (its last pull, now].
static bool async_pull_p(const ddq_step_cfg* cfg, int64_t last, int64_t now) {
  return cfg->target_period > 0 && now / cfg->target_period > last / cfg->target_period;
}

// Start of the async exchange on this ctx (any earlier steps taken, the
// replicas equal): the central model's shards start from this replica (after
// the pull at the current iteration -- a special update when it is a
// multiple of the period, e.g. 0), every worker pulled there, and the
// worker's first gradient is computed on it.
static int async_begin(ddq_ctx* c, const ddq_step_cfg* cfg) {
  const int64_t P = c->nb.L.total;
  if (!c->own) TRY(dalloc(c, &c->own, (size_t)P + kShardPad));
  if (!c->pown) TRY(dalloc(c, &c->pown, (size_t)P + kShardPad));
  if (!c->grad_ev) {
    HIP_TRY(c, hipEventCreateWithFlags(&c->grad_ev, hipEventDisableTiming));
    HIP_TRY(c, hipEventCreateWithFlags(&c->tick_ev, hipEventDisableTiming));
  }
  TRY(initial_target_sync(c, cfg));
  HIP_TRY(c, hipMemcpyAsync(c->own, c->nb.theta[0], P * 4, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(c, hipMemcpyAsync(c->pown, c->nb.theta[1], P * 4, hipMemcpyDeviceToDevice, c->stream));
  c->last_pull.assign(c->nranks, c->applied);
  c->async_on = true;
  // the owner duties run on the comm stream: it starts after the copies
  HIP_TRY(c, hipEventRecord(c->cev[0], c->stream));
  HIP_TRY(c, hipStreamWaitEvent(c->cs, c->cev[0], 0));
  return async_compute(c, cfg);
}

// Owner side of a tick, on the comm stream: the received slice (in gsl)
// applied to the owned shard on arrival (iteration += 1, the launch's own
// bookkeeping), and the central P shard updated when this tick's pull (at
// iteration it) is a special update.
// own: the push is this rank's own gradient -- applied from the gradient
// buffer in place (no copy to gsl), and the worker's copy of the shard written
// beside the central one (no pull copy)
// -- and, from the same values, that shard's kernel layouts and (on a tick that
// updates the central P) the worker's P shard and its layouts: the worker's
// refreshes after the pull skip the shard (async_after_pull)
static bool async_p_now(const ddq_step_cfg* cfg, int64_t it) {
  return cfg->target_period > 0 && it % cfg->target_period == 0;
}

// draw: the launch also draws + gathers the worker's next minibatch (B <=
// 256; the caller ordered every ctx-stream op before it, and the worker's
// compute after it), as async_compute's draw launch would
static int async_owner_apply(ddq_ctx* c, const ddq_step_cfg* cfg, int64_t it, bool own,
                             bool draw = false) {
  const ddq_update_cfg& u = cfg->update;
  const int64_t L = c->shard_len, off = (int64_t)c->rank * L;
  // (the apply kernel indexes the gradient slice from the shard's start)
  const float* g = own ? c->nb.grad + off : c->gsl;
  Prefetch pf{};
  if (draw)
    pf = make_prefetch(c->nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                       cfg->seed);
  HIP_TRY(c, launch_apply_shard(c->nb, u.rule, u.lr, u.decay, u.eps, u.momentum, u.weight_decay,
                                g, off, L, L, 1, c->cs, c->own, c->applied == 0 ? 1 : 0,
                                draw ? &pf : nullptr, own ? c->nb.theta[0] : nullptr,
                                own ? (async_p_now(cfg, it) ? 2 : 1) : 0));
  if (async_p_now(cfg, it))
    HIP_TRY(c, hipMemcpyAsync(c->pown + off, c->own + off, L * 4, hipMemcpyDeviceToDevice, c->cs));
  return DDQ_OK;
}

// Worker side after its pull (theta[0], and theta[1] when pull_p, hold the
// central model; the ctx stream waited for them): kernel layouts of Q (and
// P), then the next gradient.  own: the worker's own shard was refreshed by
// its owner apply (Q; P too when this tick updated the central P: p_own).
static int async_after_pull(ddq_ctx* c, const ddq_step_cfg* cfg, bool pull_p, bool own = false,
                            bool p_own = false, bool drawn = false) {
  const int64_t lo = own ? (int64_t)c->rank * c->shard_len : 0;
  const int64_t hi = own ? lo + c->shard_len : 0;
  p_own = p_own && own;
  HIP_TRY(c, launch_refresh(c->nb, c->stream, 0, lo, hi));
  if (pull_p) {   // P's layouts from the pulled P weights
    NetBuffers pb = c->nb;
    pb.theta[0] = c->nb.theta[1]; pb.wks[0] = c->nb.wks[1];
    HIP_TRY(c, launch_refresh(pb, c->stream, 0, p_own ? lo : 0, p_own ? hi : 0));
  }
  return async_compute(c, cfg, drawn);
}

// Host bookkeeping of a tick (every rank / member: the same tick sequence).
static void async_advance(ddq_ctx* c, int w, int64_t it) {
  c->applied = it;
  c->last_pull[w] = it;
  c->async_ticks++;
}

// One tick over RCCL (worker w pushes): point-to-point pushes / pulls and the
// owner apply on the comm stream, the pulling worker's next gradient on its
// ctx stream -- it overlaps the later ticks' owner duties.
static int rccl_async_tick(ddq_ctx* c, const ddq_step_cfg* cfg, int w) {
  const int W = c->nranks, r = c->rank;
  const int64_t L = c->shard_len;
  NetBuffers& nb = c->nb;
  const int64_t it = c->applied + 1;    // iteration after this tick's apply
  const bool pull_p = async_pull_p(cfg, c->last_pull[w], it);
  // the own push's owner apply draws + gathers this worker's next minibatch:
  // it follows everything on the ctx stream so far (the gradient, and any
  // replay insert enqueued since), not only grad_ev
  const bool draw = r == w && nb.B <= 256;
  if (draw) {
    HIP_TRY(c, hipEventRecord(c->cev[0], c->stream));
    HIP_TRY(c, hipStreamWaitEvent(c->cs, c->cev[0], 0));
  } else if (r == w && (!c->acapture || c->grad_ev_captured)) {
    HIP_TRY(c, hipStreamWaitEvent(c->cs, c->grad_ev, 0));
  }
  // push: worker w's gradient slices to their owners
  if (W > 1) {
    NCCL_TRY(c, ncclGroupStart());
    if (r == w) {
      for (int j = 0; j < W; ++j)
        if (j != r) NCCL_TRY(c, ncclSend(nb.grad + (size_t)j * L, L, ncclFloat, j, c->comm, c->cs));
    } else {
      NCCL_TRY(c, ncclRecv(c->gsl, L, ncclFloat, w, c->comm, c->cs));
    }
    NCCL_TRY(c, ncclGroupEnd());
  }
  TRY(async_owner_apply(c, cfg, it, r == w, draw));
  // pull: the owners' shards to worker w
  if (W > 1) {
    NCCL_TRY(c, ncclGroupStart());
    if (r != w) {
      NCCL_TRY(c, ncclSend(c->own + (size_t)r * L, L, ncclFloat, w, c->comm, c->cs));
      if (pull_p) NCCL_TRY(c, ncclSend(c->pown + (size_t)r * L, L, ncclFloat, w, c->comm, c->cs));
    } else {
      for (int j = 0; j < W; ++j) {
        if (j == r) continue;
        NCCL_TRY(c, ncclRecv(nb.theta[0] + (size_t)j * L, L, ncclFloat, j, c->comm, c->cs));
        if (pull_p)
          NCCL_TRY(c, ncclRecv(nb.theta[1] + (size_t)j * L, L, ncclFloat, j, c->comm, c->cs));
      }
    }
    NCCL_TRY(c, ncclGroupEnd());
  }
  if (r == w) {   // (the own shard of theta[0]: written by the owner apply;
                  // of theta[1] too when this tick updated the central P)
    const bool p_own = async_p_now(cfg, it);
    if (pull_p && !p_own)
      HIP_TRY(c, hipMemcpyAsync(nb.theta[1] + (size_t)r * L, c->pown + (size_t)r * L, L * 4,
                                hipMemcpyDeviceToDevice, c->cs));
    HIP_TRY(c, hipEventRecord(c->tick_ev, c->cs));
    HIP_TRY(c, hipStreamWaitEvent(c->stream, c->tick_ev, 0));
    TRY(async_after_pull(c, cfg, pull_p, true, p_own, draw));
  }
  async_advance(c, w, it);
  return DDQ_OK;
}

// the ctx stream waits for the comm stream's owner duties so far
static int async_join(ddq_ctx* c) {
  HIP_TRY(c, hipEventRecord(c->cev[1], c->cs));
  HIP_TRY(c, hipStreamWaitEvent(c->stream, c->cev[1], 0));
  return DDQ_OK;
}

static int async_prepare(ddq_ctx* c, const ddq_step_cfg* cfg) {
  if (c->local) return fail(c, DDQ_ESTATE, "in-process group members step with ddq_group_step");
  if (!c->cs) TRY(setup_shards(c, c->nranks));
  if (!c->async_on) TRY(async_begin(c, cfg));
  return DDQ_OK;
}

// One round-robin round (W ticks, worker 0 .. W-1): a step of the async exchange.
static int rccl_async_round(ddq_ctx* c, const ddq_step_cfg* cfg) {
  for (int w = 0; w < c->nranks; ++w) TRY(rccl_async_tick(c, cfg, w));
  return async_join(c);   // the step ends when this rank's owner duties are done
}

int ddq_async_begin(ddq_ctx* c, const ddq_step_cfg* cfg) {
  TRY(check_step(c, cfg));
  if (cfg->exchange != DDQ_EXCHANGE_ASYNC) return fail(c, DDQ_EINVAL, "cfg exchange is not async");
  TRY(set_dev(c));
  return async_prepare(c, cfg);
}

// Is this worker's gradient pushable: computed (grad_ev), and -- for an
// emulated straggler -- straggle_us of host time since that was first seen.
static int grad_ready(ddq_ctx* c, bool* ready) {
  const hipError_t e = hipEventQuery(c->grad_ev);
  if (e != hipSuccess && e != hipErrorNotReady)
    return fail(c, DDQ_EHIP, "hipEventQuery: %s", hipGetErrorString(e));
  *ready = false;
  if (e != hipSuccess) return DDQ_OK;
  const auto now = std::chrono::steady_clock::now();
  if (!c->ready_seen) {
    c->ready_seen = true;
    c->ready_at = now;
  }
  *ready = now - c->ready_at >= std::chrono::microseconds(c->straggle_us);
  return DDQ_OK;
}

int ddq_async_ready(ddq_ctx* c, int32_t* ready) {
  if (!c || !ready) return fail(c, DDQ_EINVAL, "null argument");
  if (!c->async_on) return fail(c, DDQ_ESTATE, "async exchange not begun (ddq_async_begin)");
  TRY(set_dev(c));
  bool r = false;
  TRY(grad_ready(c, &r));
  *ready = r ? 1 : 0;
  return DDQ_OK;
}

static int after_async_graph(ddq_ctx* c);

// This rank's own tick (worker == rank) as a graph.  Its launches depend on
// the host state only through whether this tick pulls P and whether its
// iteration is a special update (and the first apply of all: eager), so two
// bits pick the graph; the capture leaves the host bookkeeping as it was.
static int ensure_tick_graph(ddq_ctx* c, const ddq_step_cfg* cfg, int key) {
  if (memcmp(&c->tcfg, cfg, sizeof(*cfg)) != 0) {
    for (auto& g : c->tgexec)
      if (g) { hipGraphExecDestroy(g); g = nullptr; }
    c->tcfg = *cfg;
  }
  if (c->tgexec[key]) return DDQ_OK;
  const int64_t applied = c->applied, ticks = c->async_ticks;
  const std::vector<int64_t> last = c->last_pull;
  HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  c->acapture = true;
  c->grad_ev_captured = false;
  int rc = DDQ_OK;
  hipError_t e = hipEventRecord(c->cev[0], c->stream);   // the comm stream joins
  if (e == hipSuccess) e = hipStreamWaitEvent(c->cs, c->cev[0], 0);
  if (e != hipSuccess) rc = fail(c, DDQ_EHIP, "tick graph fork: %s", hipGetErrorString(e));
  if (rc == DDQ_OK) rc = rccl_async_tick(c, cfg, c->rank);
  hipGraph_t g = nullptr;
  e = hipStreamEndCapture(c->stream, &g);
  c->acapture = false;
  c->applied = applied;
  c->async_ticks = ticks;
  c->last_pull = last;
  if (rc != DDQ_OK) { if (g) hipGraphDestroy(g); return rc; }
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
  e = hipGraphInstantiate(&c->tgexec[key], g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
  HIP_TRY(c, hipGraphUpload(c->tgexec[key], c->stream));
  return DDQ_OK;
}

int ddq_async_tick(ddq_ctx* c, const ddq_step_cfg* cfg, int32_t worker) {
  TRY(check_step(c, cfg));
  if (cfg->exchange != DDQ_EXCHANGE_ASYNC) return fail(c, DDQ_EINVAL, "cfg exchange is not async");
  if (worker < 0 || worker >= c->nranks)
    return fail(c, DDQ_EINVAL, "worker %d out of [0, %d)", worker, c->nranks);
  TRY(set_dev(c));
  TRY(async_prepare(c, cfg));
  c->rr_rounds = 0;   // the round-robin graph's steady state no longer holds
  // this rank's own ticks (the heavy ones: its next gradient) replay a graph;
  // the other workers' ticks (a receive, the owner apply, a send) stay eager
  if (worker == c->rank && c->applied > 0) {
    const int64_t it = c->applied + 1;
    const bool pull_p = async_pull_p(cfg, c->last_pull[worker], it);
    const bool special = cfg->target_period > 0 && it % cfg->target_period == 0;
    const int key = (pull_p ? 2 : 0) | (special ? 1 : 0);
    TRY(ensure_tick_graph(c, cfg, key));
    HIP_TRY(c, hipGraphLaunch(c->tgexec[key], c->stream));
    TRY(after_async_graph(c));
    async_advance(c, worker, it);
    return DDQ_OK;
  }
  return rccl_async_tick(c, cfg, worker);
}

// ---- round-robin rounds as hipGraphs ----
// A round's launches depend on the host state only through the iteration's
// residue mod the special-update period (which ticks pull P, which owners
// copy Q -> P) and the workers' last pulls, which after one whole round-robin
// round are one round back for everyone.  So K = period / gcd(W, period)
// rounds (K W iterations, a multiple of the period) form a graph that is
// valid whenever a round starts at the residue it was captured at; the host
// bookkeeping of a replay is the captured ticks' (async_advance).  Rounds
// before that alignment (and the remainder of a call) run eagerly.
static constexpr int kAsyncGraphMaxRounds = 16;

static int async_graph_rounds(const ddq_ctx* c, const ddq_step_cfg* cfg) {
  if (cfg->target_period <= 0) return 1;
  int a = c->nranks, b = cfg->target_period;
  while (b) { const int t = a % b; a = b; b = t; }
  return cfg->target_period / a;
}

static int64_t async_phase(const ddq_ctx* c, const ddq_step_cfg* cfg) {
  return cfg->target_period > 0 ? c->applied % cfg->target_period : 0;
}

static int async_round_eager(ddq_ctx* c, const ddq_step_cfg* cfg) {
  TRY(rccl_async_round(c, cfg));
  c->steps++;
  c->rr_rounds++;
  return DDQ_OK;
}

static int ensure_async_graph(ddq_ctx* c, const ddq_step_cfg* cfg, int K) {
  if (c->agexec && memcmp(&c->acfg, cfg, sizeof(*cfg)) == 0) return DDQ_OK;
  if (c->agexec) hipGraphExecDestroy(c->agexec);
  c->agexec = nullptr;
  const int64_t applied = c->applied, ticks = c->async_ticks;
  const std::vector<int64_t> last = c->last_pull;
  HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  c->acapture = true;
  c->grad_ev_captured = false;
  // the comm stream joins the capture (its owner duties follow the graph's start)
  int rc = DDQ_OK;
  hipError_t e = hipEventRecord(c->cev[0], c->stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->cs, c->cev[0], 0);
  if (e != hipSuccess) rc = fail(c, DDQ_EHIP, "async graph fork: %s", hipGetErrorString(e));
  for (int k = 0; k < K && rc == DDQ_OK; ++k) rc = rccl_async_round(c, cfg);
  hipGraph_t g = nullptr;
  e = hipStreamEndCapture(c->stream, &g);
  c->acapture = false;
  c->applied = applied;             // the capture ran the ticks' host bookkeeping
  c->async_ticks = ticks;
  c->last_pull = last;
  if (rc != DDQ_OK) { if (g) hipGraphDestroy(g); return rc; }
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
  e = hipGraphInstantiate(&c->agexec, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
  HIP_TRY(c, hipGraphUpload(c->agexec, c->stream));
  c->acfg = *cfg;
  c->agraph_rounds = K;
  c->agraph_phase = async_phase(c, cfg);
  return DDQ_OK;
}

// After a replay of the round-robin graph: the graph's comm-stream work is a
// branch of the launch, so the comm stream itself is not ordered behind it --
// make it wait for the launch (the eager ticks / rounds that follow queue
// RCCL calls, owner applies and gsl copies on it).  A graph replay re-records
// no event either: grad_ev still marks the gradient from before the capture,
// so record it again behind the launch (whose last round computed nb.grad),
// and forget an earlier readiness observation.
static int after_async_graph(ddq_ctx* c) {
  HIP_TRY(c, hipEventRecord(c->cev[0], c->stream));
  HIP_TRY(c, hipStreamWaitEvent(c->cs, c->cev[0], 0));
  HIP_TRY(c, hipEventRecord(c->grad_ev, c->stream));
  c->ready_seen = false;
  c->grad_ev_captured = false;
  return DDQ_OK;
}

static int async_graph_steps(ddq_ctx* c, const ddq_step_cfg* cfg, int nsteps) {
  TRY(async_prepare(c, cfg));
  const int K = async_graph_rounds(c, cfg);
  int i = 0;
  if (K > kAsyncGraphMaxRounds) {
    for (; i < nsteps; ++i) TRY(async_round_eager(c, cfg));
    return DDQ_OK;
  }
  while (i < nsteps) {
    const bool steady = c->rr_rounds >= 1;
    if (steady && nsteps - i >= K &&
        (c->agexec == nullptr || memcmp(&c->acfg, cfg, sizeof(*cfg)) != 0 ||
         async_phase(c, cfg) == c->agraph_phase)) {
      TRY(ensure_async_graph(c, cfg, K));
      HIP_TRY(c, hipGraphLaunch(c->agexec, c->stream));
      TRY(after_async_graph(c));
      for (int k = 0; k < K; ++k)
        for (int w = 0; w < c->nranks; ++w) async_advance(c, w, c->applied + 1);
      c->steps += K;
      c->rr_rounds += K;
      i += K;
      continue;
    }
    TRY(async_round_eager(c, cfg));
    ++i;
  }
  return DDQ_OK;
}

int ddq_set_straggle(ddq_ctx* c, int64_t usec) {
  if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx");
  if (usec < 0 || usec > 1000000) return fail(c, DDQ_EINVAL, "usec must be in [0, 1e6]");
  c->straggle_us = usec;
  return DDQ_OK;
}

int ddq_step_async(ddq_ctx* c, const ddq_step_cfg* cfg) {
  TRY(check_step(c, cfg));
  TRY(set_dev(c));
  if (is_async(c, cfg)) {
    TRY(async_prepare(c, cfg));
    return async_round_eager(c, cfg);
  }
  TRY(check_not_async(c));
  if (c->steps == 0) TRY(initial_target_sync(c, cfg));
  c->nb.fault_k2_short = c->fault == DDQ_FAULT_MEET_TIMEOUT;   // (this step's launches only)
  c->fault = 0;
  const int rc = enqueue_step(c, cfg, nullptr, nullptr);
  c->nb.fault_k2_short = 0;
  TRY(rc);
  c->steps++;
  c->applied += step_inc(c, cfg);
  return DDQ_OK;
}

static int capture_steps(ddq_ctx* c, const ddq_step_cfg* cfg, int k, hipGraphExec_t* out) {
  HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  int rc = DDQ_OK;
  for (int i = 0; i < k && rc == DDQ_OK; ++i) rc = enqueue_step(c, cfg, nullptr, nullptr);
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(c->stream, &g);
  if (rc != DDQ_OK) { if (g) hipGraphDestroy(g); return rc; }
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
  e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
  // upload now: the first launch of a never-uploaded exec pays the upload on
  // the stream (measured ~0.3 ms in the first timed chunk otherwise)
  HIP_TRY(c, hipGraphUpload(*out, c->stream));
  return DDQ_OK;
}

// One graph holds kGraphSteps steps back to back (the launch of a graph
// costs ~9 us of device idle, measured, so it is paid once per kGraphSteps
// steps), plus a one-step graph for the remainder.  The device-side counters
// make every captured step read its own iteration / RNG state.
static constexpr int kGraphSteps = 8;

static int ensure_graph(ddq_ctx* c, const ddq_step_cfg* cfg) {
  if (is_async(c, cfg)) return DDQ_OK;   // captured when a round starts at its phase
  TRY(check_not_async(c));
  if (!c->have_graph || memcmp(&c->gcfg, cfg, sizeof(*cfg)) != 0) {
    invalidate_graph(c);
    TRY(capture_steps(c, cfg, 1, &c->gexec));
    TRY(capture_steps(c, cfg, kGraphSteps, &c->gexec_k));
    c->gcfg = *cfg;
    c->have_graph = true;
  }
  return DDQ_OK;
}

int ddq_step_graph_async(ddq_ctx* c, const ddq_step_cfg* cfg, int32_t nsteps) {
  TRY(check_step(c, cfg));
  TRY(set_dev(c));
  if (is_async(c, cfg)) return async_graph_steps(c, cfg, nsteps);
  TRY(ensure_graph(c, cfg));
  if (c->steps == 0 && nsteps > 0) TRY(initial_target_sync(c, cfg));
  int i = 0;
  for (; i + kGraphSteps <= nsteps; i += kGraphSteps)
    HIP_TRY(c, hipGraphLaunch(c->gexec_k, c->stream));
  for (; i < nsteps; ++i) HIP_TRY(c, hipGraphLaunch(c->gexec, c->stream));
  c->steps += nsteps;
  c->applied += (int64_t)nsteps * step_inc(c, cfg);
  return DDQ_OK;
}

// nsteps training steps as a chain of graph replays in which step t+1's
// sample + gather overlap step t.  Graph [p][f] trains on minibatch set p
// and (f = 1) prefetches into set 1-p; the chain starts on the parity that
// makes the LAST step train on set 0, so afterwards the ctx's minibatch,
// indices and counters are exactly those of nsteps sequential steps.
// With fused_prefetch the prefetch is extra blocks of the apply launch (no
// side stream), the first draw is the fused sample_gather kernel (which does
// not advance the counter) and every step's bookkeeping advances it, as in
// the plain graph step; chains longer than kGraphSteps + 1 replay
// kGraphSteps-step graphs (an even count: they start and end on set p).
static int capture_exec(ddq_ctx* c, hipGraphExec_t* out, const std::function<int()>& body) {
  HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  int rc = body();
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture(c->stream, &g);
  if (rc != DDQ_OK) { if (g) hipGraphDestroy(g); return rc; }
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
  e = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (e != hipSuccess) return fail(c, DDQ_EHIP, "hipGraphInstantiate: %s", hipGetErrorString(e));
  // upload now: the first launch of a never-uploaded exec pays the upload on
  // the stream (measured ~0.3 ms in the first timed chunk otherwise)
  HIP_TRY(c, hipGraphUpload(*out, c->stream));
  return DDQ_OK;
}

static int ensure_pipe(ddq_ctx* c, const ddq_step_cfg* cfg) {
  if (is_async(c, cfg))
    return fail(c, DDQ_EINVAL, "the async exchange runs round-robin rounds (ddq_step_async, "
                               "ddq_step_graph_async) or ticks (ddq_async_tick)");
  TRY(check_not_async(c));
  if (!c->mb2_state) {
    const int B = c->nb.B, S = c->nb.S;
    TRY(dalloc(c, &c->mb2_state, (size_t)B * S * S * 4));
    TRY(dalloc(c, &c->mb2_next, (size_t)B * S * S * 4));
    TRY(dalloc(c, &c->mb2_action, (size_t)B * 4));
    TRY(dalloc(c, &c->mb2_reward, (size_t)B));
    TRY(dalloc(c, &c->mb2_nonterm, (size_t)B));
    TRY(dalloc(c, &c->mb2_idx, (size_t)B));
  }
  const bool fpf = fused_prefetch(c, cfg);
  ReplayMeta* bump = fpf ? c->r_meta : nullptr;
  if (!c->have_pipe || memcmp(&c->pcfg, cfg, sizeof(*cfg)) != 0) {
    invalidate_graph(c);
    for (int p = 0; p < 2; ++p) {
      for (int f = 0; f < 2; ++f) {
        const NetBuffers cur = mb_view(c, p), nxt = mb_view(c, 1 - p);
        TRY(capture_exec(c, &c->pexec[p][f], [&]() -> int {
          return enqueue_train(c, cfg, cur, f ? &nxt : nullptr, nullptr, nullptr, bump);
        }));
      }
      if (fpf) {
        TRY(capture_exec(c, &c->pexec_k[p], [&]() -> int {
          for (int k = 0; k < kGraphSteps; ++k) {
            const int q = p ^ (k & 1);
            const NetBuffers cur = mb_view(c, q), nxt = mb_view(c, 1 - q);
            TRY(enqueue_train(c, cfg, cur, &nxt, nullptr, nullptr, bump));
          }
          return DDQ_OK;
        }));
        for (int r = 2; r <= kGraphSteps; ++r)
          TRY(capture_exec(c, &c->ptail[p][r], [&]() -> int {
            for (int k = 0; k < r; ++k) {
              const int q = p ^ (k & 1);
              const NetBuffers cur = mb_view(c, q), nxt = mb_view(c, 1 - q);
              TRY(enqueue_train(c, cfg, cur, k + 1 < r ? &nxt : nullptr, nullptr, nullptr, bump));
            }
            return DDQ_OK;
          }));
      }
    }
    c->pcfg = *cfg;
    c->have_pipe = true;
  }
  return DDQ_OK;
}

int ddq_step_prepare(ddq_ctx* c, const ddq_step_cfg* cfg, int32_t mode) {
  TRY(check_step(c, cfg));
  TRY(set_dev(c));
  if (mode == 1) return ensure_graph(c, cfg);
  if (mode == 2) return ensure_pipe(c, cfg);
  if (mode != 0) return fail(c, DDQ_EINVAL, "mode must be 0 (eager), 1 (graph) or 2 (pipelined)");
  return DDQ_OK;
}

int ddq_step_pipelined_async(ddq_ctx* c, const ddq_step_cfg* cfg, int32_t nsteps) {
  TRY(check_step(c, cfg));
  TRY(set_dev(c));
  if (nsteps <= 0) return DDQ_OK;
  TRY(ensure_pipe(c, cfg));
  const bool fpf = fused_prefetch(c, cfg);
  if (c->steps == 0) TRY(initial_target_sync(c, cfg));
  int p = (nsteps - 1) & 1;
  const NetBuffers first = mb_view(c, p);
  if (fpf) {
    HIP_TRY(c, launch_sample_gather(first, c->r_state, c->r_action, c->r_reward, c->r_nonterm,
                                    c->r_meta, cfg->seed, c->stream));
  } else {
    HIP_TRY(c, launch_sample(first, c->r_meta, cfg->seed, c->stream));
    HIP_TRY(c, launch_gather(first, c->r_state, c->r_action, c->r_reward, c->r_nonterm, c->r_meta,
                             c->stream));
  }
  for (int i = 0; i < nsteps;) {
    if (fpf && nsteps - i > kGraphSteps) {
      HIP_TRY(c, hipGraphLaunch(c->pexec_k[p], c->stream));   // ends on set p again
      c->steps += kGraphSteps;
      c->applied += (int64_t)kGraphSteps * step_inc(c, cfg);
      i += kGraphSteps;
      continue;
    }
    if (fpf && nsteps - i > 1) {   // the chain's last r steps: one graph
      const int r = nsteps - i;
      HIP_TRY(c, hipGraphLaunch(c->ptail[p][r], c->stream));
      c->steps += r;
      c->applied += (int64_t)r * step_inc(c, cfg);
      p ^= (r - 1) & 1;   // == 0: every chain ends on set 0
      i += r;
      continue;
    }
    HIP_TRY(c, hipGraphLaunch(c->pexec[p][i + 1 < nsteps ? 1 : 0], c->stream));
    c->steps++;
    c->applied += step_inc(c, cfg);
    p ^= 1;
    ++i;
  }
  return DDQ_OK;
}

// ---------------- in-process groups ----------------
int ddq_group_init(ddq_ctx** ctxs, int32_t W) {
  if (!ctxs || W < 1 || W > kMaxRanks) return fail(nullptr, DDQ_EINVAL, "bad group");
  for (int r = 0; r < W; ++r) {
    ddq_ctx* c = ctxs[r];
    if (!c) return fail(nullptr, DDQ_EINVAL, "null ctx in group");
    if (c->comm) return fail(c, DDQ_ESTATE, "ctx already has an RCCL communicator");
    if (c->nb.S != ctxs[0]->nb.S || c->nb.B != ctxs[0]->nb.B)
      return fail(c, DDQ_EINVAL, "group members must share batch and frame");
  }
  for (int r = 0; r < W; ++r) {
    ddq_ctx* c = ctxs[r];
    TRY(set_dev(c));
    c->local = true;
    c->nranks = W;
    c->rank = r;
    TRY(setup_shards(c, W));
    if (!c->gstage) TRY(dalloc(c, &c->gstage, (size_t)W * (c->nb.L.total + kShardPad)));
    invalidate_graph(c);
  }
  return DDQ_OK;
}

// In-process group ticks: rccl_async_tick with the point-to-point transfers
// as device copies, ordered by events only (no host synchronisation): owner r
// copies worker w's slice into its gsl on its comm stream once w's gradient is
// ready, applies it, and copies its shard (and P's) into w's replica -- the
// sender side of the pull, so its next apply cannot overtake the copy -- then
// marks the tick; worker w's ctx stream waits for every owner's mark, and
// recomputes.
static int group_async_tick(ddq_ctx** ctxs, int W, const ddq_step_cfg* cfg, int w) {
  ddq_ctx* cw = ctxs[w];
  const int64_t L = ctxs[0]->shard_len;
  const int64_t it = ctxs[0]->applied + 1;
  const bool pull_p = async_pull_p(cfg, ctxs[0]->last_pull[w], it);
  for (int r = 0; r < W; ++r) {
    ddq_ctx* c = ctxs[r];
    TRY(set_dev(c));
    HIP_TRY(c, hipStreamWaitEvent(c->cs, cw->grad_ev, 0));
    HIP_TRY(c, hipMemcpyAsync(c->gsl, cw->nb.grad + (size_t)r * L, L * 4,
                              hipMemcpyDeviceToDevice, c->cs));
    TRY(async_owner_apply(c, cfg, it, false));
    HIP_TRY(c, hipMemcpyAsync(cw->nb.theta[0] + (size_t)r * L, c->own + (size_t)r * L, L * 4,
                              hipMemcpyDeviceToDevice, c->cs));
    if (pull_p)
      HIP_TRY(c, hipMemcpyAsync(cw->nb.theta[1] + (size_t)r * L, c->pown + (size_t)r * L, L * 4,
                                hipMemcpyDeviceToDevice, c->cs));
    HIP_TRY(c, hipEventRecord(c->tick_ev, c->cs));
  }
  TRY(set_dev(cw));
  for (int r = 0; r < W; ++r) HIP_TRY(cw, hipStreamWaitEvent(cw->stream, ctxs[r]->tick_ev, 0));
  TRY(async_after_pull(cw, cfg, pull_p));
  for (int r = 0; r < W; ++r) async_advance(ctxs[r], w, it);
  return DDQ_OK;
}

static int group_async_prepare(ddq_ctx** ctxs, int W, const ddq_step_cfg* cfg) {
  for (int r = 0; r < W; ++r) {
    if (ctxs[r]->async_on) continue;
    TRY(set_dev(ctxs[r]));
    TRY(async_begin(ctxs[r], cfg));
  }
  return DDQ_OK;
}

static int group_sync_all(ddq_ctx** ctxs, int W) {
  for (int r = 0; r < W; ++r) {
    ddq_ctx* c = ctxs[r];
    TRY(set_dev(c));
    HIP_TRY(c, hipStreamSynchronize(c->cs));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  return DDQ_OK;
}

// One round-robin round of an in-process group (synchronised at its end).
static int group_async_round(ddq_ctx** ctxs, int W, const ddq_step_cfg* cfg) {
  TRY(group_async_prepare(ctxs, W, cfg));
  for (int w = 0; w < W; ++w) TRY(group_async_tick(ctxs, W, cfg, w));
  TRY(group_sync_all(ctxs, W));
  for (int r = 0; r < W; ++r) ctxs[r]->steps++;
  return DDQ_OK;
}

static int check_group(ddq_ctx** ctxs, int W, const ddq_step_cfg* cfg) {
  if (!ctxs || !cfg || W < 1) return fail(nullptr, DDQ_EINVAL, "bad argument");
  for (int r = 0; r < W; ++r) {
    ddq_ctx* c = ctxs[r];
    if (!c || !c->local || c->nranks != W || c->rank != r)
      return fail(c, DDQ_ESTATE, "ctx %d is not rank %d of a %d-member group", r, r, W);
    TRY(check_step(c, cfg));
  }
  return DDQ_OK;
}

// Ticks in a given worker order (deterministic: the order of a ticket run, or
// any test schedule), synchronised at the end.
int ddq_group_async_ticks(ddq_ctx** ctxs, int32_t W, const ddq_step_cfg* cfg, int32_t n,
                          const int32_t* order) {
  TRY(check_group(ctxs, W, cfg));
  if (cfg->exchange != DDQ_EXCHANGE_ASYNC) return fail(ctxs[0], DDQ_EINVAL, "cfg exchange is not async");
  if (n < 0 || (n > 0 && !order)) return fail(ctxs[0], DDQ_EINVAL, "bad tick order");
  for (int t = 0; t < n; ++t)
    if (order[t] < 0 || order[t] >= W)
      return fail(ctxs[0], DDQ_EINVAL, "tick %d: worker %d out of [0, %d)", t, order[t], W);
  TRY(group_async_prepare(ctxs, W, cfg));
  for (int t = 0; t < n; ++t) TRY(group_async_tick(ctxs, W, cfg, order[t]));
  return group_sync_all(ctxs, W);
}

// Ticket order (arrival order) for an in-process group: the host polls the
// members' gradient-ready events and gives the next ticket to the first
// member found ready (the scan starts after the last ticket's holder), then
// enqueues that tick.  Nothing waits on the device for a ticket: the order is
// decided on the host, as the reference's single server decides it by the
// order its HTTP handler takes modelLock (server.py:196-209).
int ddq_group_async_run(ddq_ctx** ctxs, int32_t W, const ddq_step_cfg* cfg, int32_t npush,
                        int32_t* order) {
  TRY(check_group(ctxs, W, cfg));
  if (cfg->exchange != DDQ_EXCHANGE_ASYNC) return fail(ctxs[0], DDQ_EINVAL, "cfg exchange is not async");
  if (npush < 0) return fail(ctxs[0], DDQ_EINVAL, "npush must be >= 0");
  TRY(group_async_prepare(ctxs, W, cfg));
  int start = 0;
  for (int t = 0; t < npush; ++t) {
    int pick = -1;
    for (int64_t spin = 0; pick < 0; ++spin) {
      for (int k = 0; k < W && pick < 0; ++k) {
        const int w = (start + k) % W;
        TRY(set_dev(ctxs[w]));
        bool r = false;
        TRY(grad_ready(ctxs[w], &r));
        if (r) pick = w;
      }
      if (pick < 0) {
        if (spin > 2000000)   // ~minutes without any gradient finishing: a stall
          return fail(ctxs[0], DDQ_EHIP, "async run: no gradient became ready");
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
    if (order) order[t] = pick;
    TRY(group_async_tick(ctxs, W, cfg, pick));
    start = (pick + 1) % W;
  }
  return group_sync_all(ctxs, W);
}

// One synchronous data-parallel step of an in-process group: the same
// kernels and exchange semantics as RCCL ranks, with the collectives done as
// device copies between the members' buffers, phase by phase.
int ddq_group_step(ddq_ctx** ctxs, int32_t W, const ddq_step_cfg* cfg) {
  TRY(check_group(ctxs, W, cfg));
  const int ex = cfg->exchange;
  if (ex == DDQ_EXCHANGE_ASYNC) return group_async_round(ctxs, W, cfg);
  for (int r = 0; r < W; ++r) TRY(check_not_async(ctxs[r]));
  const ddq_update_cfg& u = cfg->update;
  const int64_t P = ctxs[0]->nb.L.total;
  std::vector<hipEvent_t> ev(W);
  auto record_all = [&](void) -> int {
    for (int r = 0; r < W; ++r) {
      ddq_ctx* c = ctxs[r];
      TRY(set_dev(c));
      if (ev[r] == nullptr) HIP_TRY(c, hipEventCreateWithFlags(&ev[r], hipEventDisableTiming));
      HIP_TRY(c, hipEventRecord(ev[r], c->stream));
    }
    return DDQ_OK;
  };
  auto wait_all = [&](ddq_ctx* c) -> int {
    for (int j = 0; j < W; ++j) HIP_TRY(c, hipStreamWaitEvent(c->stream, ev[j], 0));
    return DDQ_OK;
  };
  int rc = [&]() -> int {
    // phase 1: sample + gather + forward/backward (+ bookkeeping) per member
    for (int r = 0; r < W; ++r) {
      ddq_ctx* c = ctxs[r];
      TRY(set_dev(c));
      if (c->steps == 0) TRY(initial_target_sync(c, cfg));
      NetBuffers nb = c->nb;
      nb.book_inc = step_inc(c, cfg);
      ReplayMeta* bump = nullptr;
      if (nb.B <= 256) {
        HIP_TRY(c, launch_sample_gather(nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm,
                                        c->r_meta, cfg->seed, c->stream));
        bump = c->r_meta;
      } else {
        HIP_TRY(c, launch_sample(nb, c->r_meta, cfg->seed, c->stream));
        HIP_TRY(c, launch_gather(nb, c->r_state, c->r_action, c->r_reward, c->r_nonterm,
                                 c->r_meta, c->stream));
      }
      TRY(enqueue_fwd_bwd_x(c, nb, nullptr, nullptr,
                            cfg->target_period > 0 ? cfg->target_period : 0, bump, false));
    }
    TRY(record_all());
    // phase 2: exchange + (owner) apply
    for (int r = 0; r < W; ++r) {
      ddq_ctx* c = ctxs[r];
      TRY(set_dev(c));
      TRY(wait_all(c));
      const NetBuffers& nb = c->nb;
      const int64_t len = c->shard_len;
      if (ex == DDQ_EXCHANGE_NONE) {
        HIP_TRY(c, launch_apply(nb, u.rule, u.lr, u.decay, u.eps, u.momentum, u.weight_decay,
                                cfg->target_period, true, c->stream));
        continue;
      }
      if (ex == DDQ_EXCHANGE_ALLREDUCE) {   // gather every gradient first (summed below)
        for (int j = 0; j < W; ++j)
          HIP_TRY(c, hipMemcpyAsync(c->gstage + (size_t)j * P, ctxs[j]->nb.grad, P * 4,
                                    hipMemcpyDeviceToDevice, c->stream));
        continue;
      }
      for (int j = 0; j < W; ++j)
        HIP_TRY(c, hipMemcpyAsync(c->gsl + (size_t)j * len, ctxs[j]->nb.grad + (size_t)r * len,
                                  len * 4, hipMemcpyDeviceToDevice, c->stream));
      int nsl = W;
      if (ex == DDQ_EXCHANGE_SHARDED) {
        HIP_TRY(c, launch_sum_slices(c->gsl, c->gsl, W, len, len, c->stream));
        nsl = 1;
      }
      HIP_TRY(c, launch_apply_shard(nb, u.rule, u.lr, u.decay, u.eps, u.momentum, u.weight_decay,
                                    c->gsl, (int64_t)r * len, len, len, nsl, c->stream));
    }
    if (ex == DDQ_EXCHANGE_ALLREDUCE) {
      TRY(record_all());       // every member holds all W gradients: sum in rank order, apply
      for (int r = 0; r < W; ++r) {
        ddq_ctx* c = ctxs[r];
        TRY(set_dev(c));
        TRY(wait_all(c));
        HIP_TRY(c, launch_sum_slices(c->nb.grad, c->gstage, W, P, P, c->stream));
        HIP_TRY(c, launch_apply(c->nb, u.rule, u.lr, u.decay, u.eps, u.momentum, u.weight_decay,
                                cfg->target_period, true, c->stream));
      }
    }
    if (ex == DDQ_EXCHANGE_SHARDED || ex == DDQ_EXCHANGE_SERVER) {
      TRY(record_all());
      // phase 3: all-gather of the owners' shards + refresh
      for (int r = 0; r < W; ++r) {
        ddq_ctx* c = ctxs[r];
        TRY(set_dev(c));
        TRY(wait_all(c));
        const int64_t len = c->shard_len;
        for (int j = 0; j < W; ++j)
          if (j != r)
            HIP_TRY(c, hipMemcpyAsync(c->nb.theta[0] + (size_t)j * len,
                                      ctxs[j]->nb.theta[0] + (size_t)j * len, len * 4,
                                      hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(c, launch_refresh(c->nb, c->stream));
      }
    }
    for (int r = 0; r < W; ++r) {
      ddq_ctx* c = ctxs[r];
      TRY(set_dev(c));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      c->steps++;
      c->applied += step_inc(c, cfg);
    }
    return DDQ_OK;
  }();
  for (auto& e : ev)
    if (e) hipEventDestroy(e);
  return rc;
}

int64_t ddq_step_count(const ddq_ctx* c) { return c ? c->steps : -1; }

// ---------------- measurement ----------------
// A mark names the kernel launched next: arm that launch's own start / stop
// events (common.h ddq_launch).  A mark no kernel follows (an RCCL call, the
// fused step's empty "apply") is still armed at the next mark: dropped.
static void mark_settle(ddq_ctx* c) {
  if (g_ext_timing.start && !c->marks.empty()) c->marks.pop_back();   // not launched
  g_ext_timing = ExtTiming{};
}

static void mark_cb(void* arg, const char* name) {
  ddq_ctx* c = reinterpret_cast<ddq_ctx*>(arg);
  mark_settle(c);
  while (c->ev_used + 2 > c->ev_pool.size()) {
    hipEvent_t e;
    hipEventCreate(&e);
    c->ev_pool.push_back(e);
  }
  hipEvent_t e0 = c->ev_pool[c->ev_used++], e1 = c->ev_pool[c->ev_used++];
  g_ext_timing = ExtTiming{e0, e1};
  c->marks.push_back({name, e0, e1});
}

int ddq_profile_step(ddq_ctx* c, const ddq_step_cfg* cfg, char* names, float* usec, int32_t cap,
                     int32_t* n) {
  TRY(check_step(c, cfg));
  if (!n) return fail(c, DDQ_EINVAL, "null n");
  if (is_async(c, cfg)) return fail(c, DDQ_EINVAL, "profile steps take no async exchange");
  TRY(check_not_async(c));
  TRY(set_dev(c));
  c->marks.clear();
  c->ev_used = 0;
  if (c->steps == 0) TRY(initial_target_sync(c, cfg));
  g_profiling = true;
  g_unmarked = 0;
  const int rc = enqueue_step(c, cfg, mark_cb, c);
  g_profiling = false;
  mark_settle(c);
  TRY(rc);
  c->steps++;
  c->applied += step_inc(c, cfg);
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (g_unmarked)   // (the step itself ran and counts)
    return fail(c, DDQ_ESTATE, "profile: %d kernel launch(es) of the step ran without a mark "
                "(their time is in no entry)", g_unmarked);
  const int k = (int)c->marks.size();
  *n = k;
  for (int i = 0; i < k && i < cap; ++i) {
    float ms = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->marks[i].start, c->marks[i].stop));
    if (usec) usec[i] = ms * 1000.f;
    if (names) {
      memset(names + 16 * i, 0, 16);
      strncpy(names + 16 * i, c->marks[i].name.c_str(), 15);
    }
  }
  return DDQ_OK;
}

int ddq_time_layer(ddq_ctx* c, const char* name, int32_t reps, float* usec) {
  if (!c) return DDQ_EINVAL;
  if (!name || !usec || reps < 1) return fail(c, DDQ_EINVAL, "time_layer: bad arguments");
  int l = 0;
  if (!strcmp(name, "conv1_fwd")) l = 1;
  else if (!strcmp(name, "conv2_fwd")) l = 2;
  else if (!strcmp(name, "conv3_fwd")) l = 3;
  else return fail(c, DDQ_EINVAL, "time_layer: unknown layer %s", name);
  TRY(set_dev(c));
  NetBuffers nb = c->nb;
  nb.fwd_only = l;
  hipEvent_t e0, e1;
  HIP_TRY(c, hipEventCreate(&e0));
  HIP_TRY(c, hipEventCreate(&e1));
  hipError_t e = launch_forward(nb, 2, c->stream, nullptr, nullptr);   // warm
  if (e == hipSuccess) e = hipEventRecord(e0, c->stream);
  for (int i = 0; i < reps && e == hipSuccess; ++i) e = launch_forward(nb, 2, c->stream, nullptr, nullptr);
  if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  HIP_TRY(c, e);
  *usec = ms * 1000.f / reps;
  return DDQ_OK;
}

double ddq_step_flops(const ddq_ctx* c) { return c ? step_flops(c->nb.B, c->nb.S) : 0.0; }

}  // extern "C"
