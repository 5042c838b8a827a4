/*
 * ddq_hip.h -- C-ABI of libddq_hip.so, the MI355X (gfx950) implementation of
 * distributed-deep-q's data-parallel DQN training step.
 *
 * The reference's hot path sits behind pycaffe (Boost.Python -> C++ caffe::Net)
 * plus numpy/h5py/Flask host code.  Every entry point below names the reference
 * interface it replaces (file:line in defc0n1/distributed-deep-q).  The Python
 * drop-ins in distributed-deep-q_amd/ddq bind these symbols with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every function returns int: DDQ_OK (0) or a negative DDQ_E* code; no C++
 *    exception and no exit() crosses the ABI.  ddq_last_error(ctx) returns the
 *    message of the last failure on that ctx (ctx == NULL: last global error).
 *  - The library owns all device memory.  Host pointers are borrowed for the
 *    duration of the call; a call that takes host buffers copies and
 *    synchronises before returning unless its name ends in _async.  A
 *    "*_on_device" flag != 0 means the pointer is a device pointer (e.g. a
 *    torch tensor's data_ptr()) and the copy is device-to-device.
 *  - One ddq_ctx per (process, GPU), bound to one HIP stream.  Calls on one
 *    ctx must be serialised by the caller; different ctxs are independent.
 *  - Float tensors cross the ABI in the reference's Caffe shapes/orders:
 *    parameters as one flat fp32 buffer in pycaffe net.params order
 *    (Qconv1.w, Qconv1.b, ..., Q_out.b), conv W (Cout,Cin,k,k), minibatch
 *    state/next_state (B,4,S,S), action (B,4,1,1) one-hot, reward and
 *    non_terminal (B,1,1,1).  Internal device layouts are private.
 */
#ifndef DDQ_HIP_H
#define DDQ_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DDQ_ABI_VERSION 6   /* 5: ddq_step_cfg.reserved -> flags; ddq_synchronize reports a
                              small-map step's spin timeout as DDQ_ESTATE.
                              6: DDQ_STEP_REPEAT_CONV2_FWD removed (flag 2 is refused);
                              a timed-out step applies nothing; ddq_inject_fault,
                              ddq_small_path */

enum ddq_status {
  DDQ_OK = 0,
  DDQ_EINVAL = -1,   /* bad argument (sizes, names, B >= valid ...)          */
  DDQ_ENOMEM = -2,   /* device allocation failed                             */
  DDQ_EHIP = -3,     /* HIP runtime error                                    */
  DDQ_ERCCL = -4,    /* RCCL error                                           */
  DDQ_ESTATE = -5,   /* call not valid in the current state (no replay ...)  */
  DDQ_ERANGE = -6    /* data out of range (e.g. stored action >= num_actions) */
};

typedef struct ddq_ctx ddq_ctx;

/* Network description.  Replaces train_val.prototxt's MEMORY_DATA dims
 * (models/deepq/train_val.prototxt:2-37) and the GAMMA coefficient (:473). */
typedef struct ddq_net_desc {
  int32_t batch;        /* B, memory_data_param.batch_size (32)               */
  int32_t frame;        /* S, height == width (16 in deepq16); multiple of 8  */
  int32_t channels;     /* must be 4 (4-frame history, expgain.py:9)          */
  int32_t actions;      /* must be 4 (barista/constants.py:8)                 */
  float gamma;          /* 0.85 (train_val.prototxt:473)                      */
} ddq_net_desc;

/* One parameter blob of the flat layout (one tower).  Replaces iteration over
 * pycaffe net.params (messaging.py:57-66, server.py:238-244). */
typedef struct ddq_blob_desc {
  char name[16];        /* "Qconv1" ... "Q_out" (P tower: same with 'P')      */
  int32_t index;        /* 0 = weight, 1 = bias                               */
  int32_t shape[4];     /* Caffe-2014 4-D blob shape                          */
  int64_t offset;       /* element offset in the flat tower buffer            */
  int64_t count;        /* element count                                      */
} ddq_blob_desc;

/* Update rules of param-server/server.py:81-124 (+ Caffe SGDSolver momentum). */
enum ddq_rule {
  DDQ_RULE_SGD = 0,            /* server.py:81-83   theta -= lr*g             */
  DDQ_RULE_RMSPROP = 1,        /* server.py:86-105  lagged cache (default)    */
  DDQ_RULE_ADAGRAD = 2,        /* server.py:108-124                           */
  DDQ_RULE_MOMENTUM_CAFFE = 3  /* solver.prototxt:4-11 semantics (optional)   */
};

typedef struct ddq_update_cfg {
  int32_t rule;          /* enum ddq_rule                                     */
  float lr;              /* server.py:268 default 1e-4 (momentum: base_lr)    */
  float decay;           /* rmsprop decay, server.py:270 default 0.9          */
  float eps;             /* 1e-8 inside the sqrt, server.py:105,124           */
  float momentum;        /* momentum rule only (0.9)                          */
  float weight_decay;    /* momentum rule only (0.0005)                       */
} ddq_update_cfg;

/* Gradient exchange of a data-parallel step (replaces the HTTP gradient POST
 * + server apply + model GET round trip, baristanet.py:85-133,
 * server.py:181-209).  Used when the ctx has a communicator (ddq_comm_init)
 * or belongs to an in-process group (ddq_group_init); ignored otherwise. */
enum ddq_exchange {
  DDQ_EXCHANGE_NONE = 0,
  /* W gradients computed at the same theta, summed, applied once (replicated
   * apply on every rank).  Equals the server applying W equally-stale SGD
   * gradients; a documented deviation for rmsprop/adagrad. */
  DDQ_EXCHANGE_ALLREDUCE = 1,
  /* Same semantics, sharded: reduce-scatter(sum) -> each rank applies its
   * 1/W shard (optimizer state sharded) -> all-gather of theta. */
  DDQ_EXCHANGE_SHARDED = 2,
  /* Param-server semantics (server.py:196-209): every rank owns a 1/W shard
   * and its optimizer state; gradient slices go all-to-all and the owner
   * applies the W gradients one by one in rank (ticket) order, exactly as
   * the server applies gradients on arrival; iteration += W per step; then
   * all-gather of theta.  Staleness within a step: 0..W-1 updates. */
  DDQ_EXCHANGE_SERVER = 3,
  /* Asynchronous param server (server.py:181-209 with free-running workers,
   * main.py:61-112): rank r owns shard r of the central model (and its
   * optimizer state).  A TICK is one push: worker w sends the gradient it
   * computed on the model it last pulled, the owners apply it on arrival
   * (iteration += 1), worker w pulls the owners' shards (and the central P
   * tower when a special-update pull happened since its last pull) and
   * immediately computes its next gradient while later ticks proceed.  The
   * arrival order is either round-robin (the deterministic schedule: one
   * step of ddq_step_async / ddq_step_graph_async / ddq_group_step = W ticks,
   * staleness W-1) or ticket order (ddq_async_tick with the worker whose
   * gradient was ready first, ddq_group_async_run): a fast worker pushes
   * more often than a slow one, as in the reference.  Once begun on a ctx,
   * only async steps / ticks run there. */
  DDQ_EXCHANGE_ASYNC = 4
};

/* One fused training step (main.py:61-103 debug_process_connection body,
 * minus acting): sample B indices (device RNG) -> gather -> P/Q forward ->
 * Bellman target + loss -> Q backward -> [exchange] -> apply ->
 * [P <- Q when the next pull sees iteration % target_period == 0]. */
typedef struct ddq_step_cfg {
  ddq_update_cfg update;
  int32_t target_period;   /* server.py:274 --special-update (10); 0 = never */
  int32_t exchange;        /* enum ddq_exchange                              */
  uint64_t seed;           /* device index-stream seed (per rank)            */
  int32_t overlap;         /* ALLREDUCE over RCCL: reduce the fc4 weight
                              bucket on a comm stream under the conv backward */
  int32_t flags;           /* DDQ_STEP_* bits, 0 = none                      */
} ddq_step_cfg;

/* Exchange-free steps: fc4's weight gradient (96 % of the parameters) is
 * computed and applied tile by tile inside the slab-reduce launch and NOT
 * stored to the gradient buffer (8.4 MB of writes per step at 64x64), so
 * ddq_get_grads after such a step returns that block of an earlier step
 * (at S = 16 the block is stored regardless: the fused step's last launch
 * applies it from there).
 * The update is unchanged, bit for bit.  No effect on exchanged steps (their
 * gradient is what is exchanged). */
#define DDQ_STEP_NO_GRAD_STORE 1

/* ---------------- context ---------------------------------------------- */
/* caffe.Net(prototxt, model) + set_mode_gpu + set_phase_test
 * (baristanet.py:16, main.py:147-151).  Dropout is identity (TEST phase). */
int ddq_create(ddq_ctx** out, int device, const ddq_net_desc* desc);
int ddq_destroy(ddq_ctx* ctx);
const char* ddq_last_error(const ddq_ctx* ctx);
int ddq_abi_version(void);
/* Use an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream). */
int ddq_set_stream(ddq_ctx* ctx, void* hip_stream);
/* The ctx's HIP stream (e.g. for torch.cuda.ExternalStream events). */
int ddq_get_stream(const ddq_ctx* ctx, void** hip_stream);
/* Wait for the ctx's streams.  DDQ_ESTATE when a small-map (S = 16) step's
 * inter-workgroup meeting timed out since the last call.  The launches went
 * on (no hang) but wrote no parameter, optimizer state, P copy or iteration
 * from that step on (a fused-apply step; an exchanged step's gradient is
 * invalid); this call clears the flag, restarts the meeting counters and
 * takes the device iteration back, so the ctx steps on from the last good
 * update. */
int ddq_synchronize(ddq_ctx* ctx);

/* Failpoints for the error paths' tests (no reference counterpart). */
enum ddq_fault {
  DDQ_FAULT_NONE = 0,          /* disarm                                        */
  /* the next eager step (ddq_step_async) launches its fc4 chain one workgroup
   * short, so the fan-in meeting times out: ddq_synchronize must then return
   * DDQ_ESTATE with the model unchanged.  Small-map ctxs only (DDQ_ESTATE
   * otherwise). */
  DDQ_FAULT_MEET_TIMEOUT = 1
};
int ddq_inject_fault(ddq_ctx* ctx, int32_t fault);

/* 1 when the ctx runs the four-launch small-map step (S = 16, B <= 256, and
 * every meeting launch's workgroups fit the device at once: checked with the
 * occupancy API at ddq_create), 0 when it runs the general kernels; why
 * (nullable, cap bytes) receives the reason it is off. */
int ddq_small_path(const ddq_ctx* ctx, char* why, int32_t cap);

/* ---------------- parameters ------------------------------------------- */
/* Number of fp32 parameters of ONE tower (228,132 at S=16,
 * results/cost-vs-image-size.txt:2). */
int64_t ddq_num_params(const ddq_ctx* ctx);
/* net.params names/shapes/offsets (Q tower; P identical with prefix 'P'). */
int ddq_param_layout(const ddq_ctx* ctx, ddq_blob_desc* out, int32_t cap, int32_t* n);
/* .data / .diff .flat[:] access (messaging.py:66,111).  which: 0 = Q, 1 = P. */
int ddq_set_params(ddq_ctx* ctx, int32_t which, const float* src, int64_t n, int32_t src_on_device);
int ddq_get_params(ddq_ctx* ctx, int32_t which, float* dst, int64_t n, int32_t dst_on_device);
int ddq_get_grads(ddq_ctx* ctx, float* dst, int64_t n, int32_t dst_on_device);
int ddq_set_grads(ddq_ctx* ctx, const float* src, int64_t n, int32_t src_on_device);
/* special_update_transform_model (server.py:127-137): P <- Q. */
int ddq_sync_target(ddq_ctx* ctx);

/* ---------------- replay (replay.py) ----------------------------------- */
/* ReplayDataset.__init__ storage (replay.py:48-61), HBM resident, zeroed. */
int ddq_replay_create(ddq_ctx* ctx, int64_t capacity);
/* add_experience (replay.py:70-92); state == NULL marks a terminal step and
 * leaves the slot stale.  state: 4*S*S uint8 (C,H,W). */
int ddq_replay_add(ddq_ctx* ctx, int32_t action, int32_t reward, const uint8_t* state);
int ddq_replay_info(const ddq_ctx* ctx, int64_t* head, int64_t* valid, int64_t* capacity);
/* Bulk load / store of the ring (the HDF5 datasets of replay.py:48-61,
 * persisted by __del__ :185-192). */
int ddq_replay_import(ddq_ctx* ctx, const uint8_t* state, const uint8_t* action,
                      const int16_t* reward, const uint8_t* non_terminal,
                      int64_t n, int64_t head, int64_t valid);
int ddq_replay_export(ddq_ctx* ctx, uint8_t* state, uint8_t* action, int16_t* reward,
                      uint8_t* non_terminal, int64_t n);
/* sample_direct (replay.py:144-183) given the sorted index list the host
 * drew (replay.py:152-159): assembles the device minibatch bit-exactly.
 * Returns DDQ_EINVAL if B >= valid (replay.py:147-150). */
int ddq_replay_sample(ddq_ctx* ctx, const int32_t* sorted_idx, int32_t batch);
/* Device-RNG draw of B distinct indices in [0,valid) \ {head-1}, sorted,
 * then the same gather (perf mode).  Enqueued, no sync. */
int ddq_replay_sample_device_async(ddq_ctx* ctx, uint64_t seed);
/* Copy the current device minibatch out in Caffe shapes (baristanet.py:30-34). */
int ddq_read_minibatch(ddq_ctx* ctx, float* state, float* action, float* reward,
                       float* next_state, float* non_terminal);
/* Set the minibatch directly (set_input_arrays binding, baristanet.py:41-43;
 * dummy_load_minibatch :70-83). */
int ddq_write_minibatch(ddq_ctx* ctx, const float* state, const float* action,
                        const float* reward, const float* next_state,
                        const float* non_terminal);
/* Fill the whole ring by tiling `pool` transitions (slot i <- pool entry
 * i % pool) on the device, then set head/valid: the 1M-slot HBM replay of
 * SURVEY 8(d) C5 without a 16 GB host image.  Host arrays of `pool` entries. */
int ddq_replay_fill_tiled(ddq_ctx* ctx, const uint8_t* state, const uint8_t* action,
                          const int16_t* reward, const uint8_t* non_terminal, int64_t pool,
                          int64_t head, int64_t valid);
/* Large-batch sample_direct (replay.py:144-183) for n <= valid/2 (any n, not
 * tied to the net batch): device draw of n distinct indices uniform over
 * [0,valid) \ {head-1}, sorted, written to idx; then s <- S[idx],
 * s' <- S[idx+1] (N-1 wraps to 0) as f32 (n,4,S,S), one-hot action (n,4),
 * reward (n), non_terminal (n) of idx+1.  ALL pointers are device pointers
 * (e.g. torch tensors).  The first call allocates the sampler's bitmap
 * (capacity/8 bytes).  Enqueued, no sync; ddq_replay_status reports a
 * stored action >= 4 or a failed draw. */
int ddq_replay_sample_batch_async(ddq_ctx* ctx, int32_t n, uint64_t seed, int32_t* idx,
                                  float* state, float* action, float* reward,
                                  float* next_state, float* non_terminal);
/* The same Caffe-layout gather for a caller-given sorted index list (device). */
int ddq_replay_gather_batch_async(ddq_ctx* ctx, const int32_t* idx, int32_t n, float* state,
                                  float* action, float* reward, float* next_state,
                                  float* non_terminal);
/* Synchronise and report (then clear) the replay's sticky device error flag. */
int ddq_replay_status(ddq_ctx* ctx);
/* Last sorted index list used by the gather (device -> host). */
int ddq_read_indices(ddq_ctx* ctx, int32_t* idx, int32_t batch);
/* Device index draws made so far (the device RNG stream position; reset by
 * ddq_replay_create).  Draw d is the minibatch of the (d+1)-th device-drawn
 * step of this ctx. */
int ddq_replay_draws(ddq_ctx* ctx, int64_t* draws);
/* Debug / parity log of the device draws: every device-drawn sorted index
 * set d (sample kernels, fused step draws, pipelined prefetches) is also
 * written to a device ring of `draws` entries of B int32 (0 disables).  Lets a
 * checker replay exactly the minibatches a graph-captured chain trained on
 * (the role of replay.py:152-159's host index list).  Invalidates graphs. */
int ddq_index_log_enable(ddq_ctx* ctx, int64_t draws);
/* Copy draws [first, first+n) (each B sorted int32) out of the log; they must
 * be among the last `draws` made. */
int ddq_index_log_read(ddq_ctx* ctx, int64_t first, int64_t n, int32_t* out);

/* ---------------- compute ---------------------------------------------- */
/* net.forward(); net.backward() (baristanet.py:138-140).  loss may be NULL. */
int ddq_forward_backward(ddq_ctx* ctx, float* loss);
int ddq_forward_backward_async(ddq_ctx* ctx);
/* forward(end='Q_out') over the bound minibatch (baristanet.py:144). */
int ddq_forward_q(ddq_ctx* ctx);
/* net.blobs[name].data for name in {"Q_out","P_out","Q_sa","P_sa",
 * "target_Q_sa","loss"} (B*4, B*4, B, B, B, 1 floats). */
int ddq_read_blob(ddq_ctx* ctx, const char* name, float* dst, int64_t n);
/* Argmax/ReLU routing bytes of pool layer 1..3 of the Q tower for the last
 * forward_backward, in Caffe (B,C,H/2,W/2) order: 0..3 = first-max position
 * in the 2x2 window (row-major), 4 = window max <= 0 (no gradient). */
int ddq_read_pool_mask(ddq_ctx* ctx, int32_t layer, uint8_t* dst, int64_t n);
/* select_action (baristanet.py:142-146) for n states (n <= B, uint8 C,H,W):
 * argmax_a Q(s,a), first max wins.  Does not touch the bound minibatch. */
int ddq_select_action(ddq_ctx* ctx, const uint8_t* states, int32_t n, int32_t* actions);

/* ---------------- apply (param server) --------------------------------- */
/* apply_descent + update_fn (server.py:49-124) on the Q tower with the
 * current gradient buffer.  Optimizer state lives on device. */
int ddq_apply(ddq_ctx* ctx, const ddq_update_cfg* cfg);
int ddq_apply_async(ddq_ctx* ctx, const ddq_update_cfg* cfg);
/* Forget rmsprop/adagrad/momentum state (server.py:229-231 clear()). */
int ddq_reset_optimizer(ddq_ctx* ctx);
int ddq_get_optimizer_state(ddq_ctx* ctx, float* dst, int64_t n);

/* ---------------- communication (RCCL over xGMI) ----------------------- */
/* Replace the HTTP/Redis gradient round trip (baristanet.py:105-123,
 * server.py:196-209) with a sum all-reduce of the flat gradient buffer. */
int ddq_comm_get_unique_id(uint8_t id[128]);
int ddq_comm_init(ddq_ctx* ctx, const uint8_t id[128], int32_t nranks, int32_t rank);
int ddq_allreduce_grads(ddq_ctx* ctx);
int ddq_allreduce_grads_async(ddq_ctx* ctx);

/* ---------------- fused step + graphs ---------------------------------- */
int ddq_step_async(ddq_ctx* ctx, const ddq_step_cfg* cfg);
/* Capture one step into a hipGraph (re-captured when cfg changes) and replay
 * it nsteps times back to back.  Enqueued, no sync. */
int ddq_step_graph_async(ddq_ctx* ctx, const ddq_step_cfg* cfg, int32_t nsteps);
/* nsteps steps as graph replays with step t+1's replay sample + gather
 * overlapped with step t (double-buffered minibatch).  Same results, indices
 * and counters as nsteps sequential ddq_step_async calls.  Enqueued, no sync. */
int ddq_step_pipelined_async(ddq_ctx* ctx, const ddq_step_cfg* cfg, int32_t nsteps);
/* Capture + instantiate (and upload) the graphs of a step mode without
 * launching anything: mode 0 = eager (no-op), 1 = ddq_step_graph_async,
 * 2 = ddq_step_pipelined_async.  Lets multi-rank callers agree on a mode
 * (every rank prepared it) before any rank enters a collective. */
int ddq_step_prepare(ddq_ctx* ctx, const ddq_step_cfg* cfg, int32_t mode);
/* In-process data parallelism: W ctxs (W workers sharing a GPU, or peer-
 * enabled devices) exchange through device copies instead of RCCL, with the
 * same exchanges, shard layout and kernels as ddq_comm_init ranks.  The
 * group step is synchronous and runs phase by phase over the members. */
int ddq_group_init(ddq_ctx** ctxs, int32_t nranks);
int ddq_group_step(ddq_ctx** ctxs, int32_t nranks, const ddq_step_cfg* cfg);
/* Steps taken so far (drives the target-sync period). */
int64_t ddq_step_count(const ddq_ctx* ctx);

/* ---------------- asynchronous param server in arrival order ------------ */
/* (DDQ_EXCHANGE_ASYNC, server.py:196-209 applying pushes as they arrive.)
 * ddq_async_begin: the central model's shards start from this replica and the
 * worker computes its first gradient (implicit in the calls below).
 * ddq_async_ready: *ready = 1 once this worker's gradient is computed (it may
 * take the next ticket).  ddq_async_tick: enqueue tick `worker` -- every rank
 * calls it with the same worker sequence (the tickets, e.g. from a TCP store:
 * ddq/dist.py AsyncTicketLoop); enqueued, no sync (ddq_synchronize waits for
 * the owner duties too). */
int ddq_async_begin(ddq_ctx* ctx, const ddq_step_cfg* cfg);
int ddq_async_ready(ddq_ctx* ctx, int32_t* ready);
int ddq_async_tick(ddq_ctx* ctx, const ddq_step_cfg* cfg, int32_t worker);
/* In-process group in ticket order: npush ticks, each given to the first
 * member (after the previous ticket's holder) whose gradient is ready, polled
 * on the host; order[t] (nullable) receives tick t's worker.  Synchronous. */
int ddq_group_async_run(ddq_ctx** ctxs, int32_t nranks, const ddq_step_cfg* cfg, int32_t npush,
                        int32_t* order);
/* The same ticks in a given worker order (deterministic replay of a ticket
 * run, or any schedule).  Synchronous. */
int ddq_group_async_ticks(ddq_ctx** ctxs, int32_t nranks, const ddq_step_cfg* cfg, int32_t n,
                          const int32_t* order);
/* Straggler emulation (fault injection, cf. the dummy driver's injected
 * failures, baristanet.py:125-133): every gradient this worker computes
 * becomes pushable (ddq_async_ready, ticket runs) usec of host time after it
 * is computed -- a slow worker loop, without occupying the GPU.  0 disables. */
int ddq_set_straggle(ddq_ctx* ctx, int64_t usec);

/* ---------------- measurement ------------------------------------------ */
/* Kernel ids for ddq_profile_step. */
#define DDQ_MAX_KERNELS 32
/* Run one eager step; every kernel is launched with start / stop events of
 * its own (hipExtLaunchKernel: the dispatch's timestamps, no marker packets
 * between the kernels); fills names (16 chars each, NUL padded) and each
 * kernel's device microseconds, in step order (RCCL calls are not timed). */
int ddq_profile_step(ddq_ctx* ctx, const ddq_step_cfg* cfg, char* names, float* usec,
                     int32_t cap, int32_t* n);
/* Launch one forward conv layer ("conv1_fwd", "conv2_fwd" or "conv3_fwd",
 * both towers, the step's own kernel and arguments) reps times back to back
 * between two HIP events on the ctx stream; *usec = average device time per
 * launch (no per-launch event overhead: the roofline's kernel time). */
int ddq_time_layer(ddq_ctx* ctx, const char* name, int32_t reps, float* usec);
/* Algorithmic FLOPs of one step (SURVEY.md 8(d) model, for the roofline). */
double ddq_step_flops(const ddq_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* DDQ_HIP_H */
