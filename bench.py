#!/usr/bin/env python3
"""Benchmark: DQN minibatch updates/sec on MI355X (BASELINE.json metric).

One step = one minibatch update of the deepq network on one GPU:
  device index draw -> replay gather -> P/Q forward -> Bellman target + loss ->
  Q backward -> [RCCL sum all-reduce of the gradient] -> rmsprop apply
  (param-server default rule) -> P <- Q every 10 updates,
captured into hipGraphs (8 steps per graph) and replayed; by default the next
step's draw + gather ride on each step's apply launch into a second minibatch
buffer (``ddq_step_pipelined_async``: bit-identical to sequential steps).  Workload at N=1: BASELINE.json
configs[1] -- deepq Snake, batch 32, 4-frame 64x64 history, 30 000-slot HBM
replay filled with synthetic Snake frames.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Prints ONE JSON line (rank 0).  ``value`` = minibatch updates/s summed over
all ranks (each rank consumes its own minibatch per step: weak scaling).
``roofline``: dominant kernel measured with HIP events on the ctx stream
(ddq_profile_step) vs the peak of the arithmetic it runs (split-bf16 kernels:
the bf16 dense peak over their products per f32 product).  ``cpu_baseline``: the oracle's C
restatement of the Caffe CPU step (oracle/libddq_cpu.so) timed on the host
cores on a bounded sample of the same workload.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-deep-q_amd")]

METRIC = "DQN minibatch updates/sec (fwd+bwd+sync+apply) @1/2/4/8 GPU; % MFMA/HBM peak"
F32_MFMA_PEAK = 157.3e12      # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense
HBM_PEAK = 8.0e12


def kernel_flops(B, S):
    """Algorithmic FLOPs per launch of each MFMA kernel (2 * MACs)."""
    s2, s3, s4 = S // 2, S // 4, S // 8
    k4 = 64 * s4 * s4
    c1 = 2.0 * B * S * S * 32 * 196
    c2 = 2.0 * B * s2 * s2 * 64 * 800
    c3 = 2.0 * B * s3 * s3 * 64 * 576
    fc = 2.0 * B * 512 * k4
    return {"conv1_fwd": 2 * c1, "conv2_fwd": 2 * c2, "conv3_fwd": 2 * c3, "fc4_fwd": 2 * fc,
            "fc4_dgrad": fc, "fc4_wgrad": fc, "conv3_wgrad": c3, "conv3_dgrad": c3,
            "conv2_wgrad": c2, "conv2_dgrad": c2, "conv1_wgrad": c1}


# rocprof kernel symbol (prefix) of each profiled step kernel
KERNEL_SYMBOL = {
    "sample_gather": "ddq::sample_gather_kernel",
    "conv1_fwd": "void ddq::split_conv1_kernel",
    "conv2_fwd": "void ddq::split_conv_kernel<32, 32, 64, 5,",
    "conv3_fwd": "void ddq::split_conv_kernel<64, 64, 64, 3, 8, 8, 2, 2,",
    "fc4_fwd": "void ddq::fc4_fwd_split_kernel",
    "head": "ddq::fc4_head_kernel",
    "fc4_dgrad": "void ddq::fc4_dgrad_direct_kernel",
    "fc4_wgrad": "ddq::fc4_wgrad_kernel",
    "conv3_wgrad": "void ddq::wgrads_kernel<64, 64, 3, 1",
    "conv3_dgrad": "void ddq::split_conv_kernel<64, 64, 64, 3, 4, 8,",
    "conv2_wgrad": "void ddq::wgrads_kernel<32, 64, 5, 2",
    "conv2_dgrad": "void ddq::split_conv_kernel<64, 64, 32, 5,",
    "conv1_wgrad": "void ddq::wgrad1s_kernel",
    "wgrad_reduce": "ddq::wgrad_reduce_kernel",
    "apply": "ddq::apply_kernel",
}

# How each MFMA kernel computes its f32-exact result (csrc/split.h, wgrads.h):
# "split" = operands split into three bf16 planes, 6 bf16 products per f32
# product; "split3" = one operand exact in bf16 (the frames), 3 products;
# "f32" = v_mfma_f32_32x32x2_f32 / f32 VALU.  Its roofline peak is the bf16
# dense peak over the products per f32 product (the f32 MFMA peak for "f32").
KERNEL_ARITH = {
    "conv1_fwd": "split3", "conv2_fwd": "split", "conv3_fwd": "split",
    "conv1_wgrad": "split3", "conv2_wgrad": "split", "conv3_wgrad": "split",
    "conv2_dgrad": "split", "conv3_dgrad": "split", "fc4_fwd": "split", "fc4_dgrad": "split",
    "fc4_wgrad": "f32",
}
BF16_MFMA_PEAK = 2.5e15       # MI355X_MICROARCH.md: dense bf16


def arith_peak(kernel):
    kind = KERNEL_ARITH.get(kernel, "f32")
    return {"split": BF16_MFMA_PEAK / 6, "split3": BF16_MFMA_PEAK / 3}.get(kind, F32_MFMA_PEAK)


def pmc_traffic(label, B, S):
    """HBM bytes per launch of `label` from the committed PMC summary
    (profiles/r02_pmc.json, tools/gpu/run_measure.sh: FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md gfx950 correction), valid for the bench default shape."""
    path = os.path.join(ROOT, "profiles", "r02_pmc.json")
    if (B, S) != (32, 64) or not os.path.exists(path):
        return None
    sym = KERNEL_SYMBOL.get(label)
    for name, e in json.load(open(path))["kernels"].items():
        if sym and name.startswith(sym) and "hbm_bytes" in e:
            return round(e["hbm_bytes"])
    return None


def fill_replay(net, N, S, seed):
    from ddq.expgain import synthetic_transitions
    pool = min(N, 4096)
    st, ac, rw, nt = synthetic_transitions(pool, S, seed=seed)
    reps = (N + pool - 1) // pool
    net.replay_import(np.tile(st, (reps, 1, 1, 1))[:N], np.tile(ac, reps)[:N],
                      np.tile(rw, reps)[:N], np.tile(nt, reps)[:N].astype(np.uint8), 0, N)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_updates(lib, B, S, seed, threads, budget_s, max_steps):
    """Time sample->gather->P/Q fwd->target->Q bwd->rmsprop apply updates of the
    oracle's C restatement (Caffe CPU algorithm) on `threads` OpenMP threads."""
    from oracle import ref_numpy as ref
    from ddq.expgain import synthetic_transitions
    fp = ctypes.POINTER(ctypes.c_float)
    N = 1024
    st, ac, rw, nt = synthetic_transitions(N, S, seed=seed)
    theta = ref.flatten(ref.init_params(S, seed=42))
    thetaP = theta.copy()
    cache = np.zeros_like(theta)
    grad = np.zeros_like(theta)
    rng = np.random.default_rng(seed)
    img = 4 * S * S
    P = lambda a: a.ctypes.data_as(fp)
    t0 = time.perf_counter()
    steps = 0
    while steps < max_steps and (steps == 0 or time.perf_counter() - t0 < budget_s):
        idx = ref.draw_indices(rng, N, 0, B)
        nxt = np.where(idx + 1 == N, 0, idx + 1)
        s = st[idx].astype(np.float32).reshape(B, img)
        s2 = st[nxt].astype(np.float32).reshape(B, img)
        a = np.zeros((B, 4), np.float32)
        a[np.arange(B), ac[nxt]] = 1
        r = rw[nxt].astype(np.float32)
        n = nt[nxt].astype(np.float32)
        rc = lib.ddq_cpu_full_pass(B, S, P(theta), P(thetaP), P(s), P(a), P(r), P(s2), P(n),
                                   ctypes.c_float(0.85), P(grad), None, threads)
        assert rc == 0
        lib.ddq_cpu_apply(1, ctypes.c_long(theta.size), P(theta), P(grad), P(cache),
                          int(steps == 0), ctypes.c_float(1e-4), ctypes.c_float(0.9),
                          ctypes.c_float(1e-8))
        steps += 1
    return steps, time.perf_counter() - t0


def cpu_baseline(B, S, seed, budget_s=12.0, max_steps=2000):
    """Oracle C restatement (Caffe CPU algorithm: im2col + SGEMM, fp32, OpenMP)
    of the same update step, on all host cores and on one core (BASELINE.md
    section 2), with the reference's own published 2015 Caffe CPU time for
    context (results/cost-vs-image-size.txt:4, hardware unstated)."""
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "libddq_cpu.so"))
    lib.ddq_cpu_full_pass.restype = ctypes.c_int
    lib.ddq_cpu_apply.restype = ctypes.c_int
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count()
    cores = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    lib.ddq_cpu_step_flops.restype = ctypes.c_double
    lib.ddq_cpu_set_isa.restype = ctypes.c_int
    isa = lib.ddq_cpu_set_isa(512)
    flops = lib.ddq_cpu_step_flops(B, S)
    steps, dt = _cpu_updates(lib, B, S, seed, cores, budget_s, max_steps)
    s1, d1 = _cpu_updates(lib, B, S, seed, 1, budget_s / 2, max(2, max_steps // 8))
    published = {16: 81.7, 32: 252.8, 64: 981.5, 128: 4044.0}.get(S)
    out = {"value": round(steps / dt, 4), "unit": "updates/s", "cores": cores, "kind": "port",
           "gflops": round(flops * steps / dt / 1e9, 1),
           "sample": "%d updates (sample->gather->P/Q fwd->target->Q bwd->rmsprop apply) "
                     "at B=%d, %dx%d, oracle/ddq_cpu.c: im2col + packed blocked SGEMM "
                     "(AVX%d micro-kernel) per image for the convs, batch GEMMs for fc4, "
                     "every layer once, fp32, %d OpenMP threads, %.1f s; %.2f GFLOP per update"
                     % (steps, B, S, S, isa if isa == 512 else 2, cores, dt, flops / 1e9),
           "cpu_model": cpu_model(),
           "single_core": {"value": round(s1 / d1, 4), "cores": 1,
                           "gflops": round(flops * s1 / d1 / 1e9, 1),
                           "sample": "%d updates, %.1f s" % (s1, d1)}}
    if published:
        out["reference_published"] = {
            "value": round(1000.0 / published, 4), "unit": "updates/s (fwd+bwd only)",
            "source": "results/cost-vs-image-size.txt (Caffe CPU, %.1f ms fwd+bwd at %dx%d "
                      "B=32, hardware unstated)" % (published, S, S)}
    return out


# algorithmic HBM bytes per launch of the fc4 kernels: W4 (512 x K fp32 per
# tower) plus activations in and out (K = 64 (S/8)^2)
FC4_BYTES = {
    "fc4_fwd": lambda B, S: 2 * (512 * 64 * (S // 8) ** 2 * 4 + B * 64 * (S // 8) ** 2 * 4),
    "fc4_dgrad": lambda B, S: 512 * 64 * (S // 8) ** 2 * 4 + B * 512 * 4 + B * 64 * (S // 8) ** 2 * 4,
    "fc4_wgrad": lambda B, S: 512 * 64 * (S // 8) ** 2 * 4 + B * 512 * 4 + B * 64 * (S // 8) ** 2 * 4,
}


def kernel_roofline(avg_us, B, S, P):
    """Per-kernel fraction of its roofline: conv kernels vs the
    peak of their arithmetic (arith_peak); fc4, the replay gather and the apply
    vs HBM (algorithmic bytes:
    gather 2*B*4*S^2 u8 read + f32 write; rmsprop apply 20*P, +8P on sync
    steps not counted).  Device times are the eager HIP-event times."""
    fl = kernel_flops(B, S)
    out = {}
    for k, us in avg_us.items():
        if us <= 0:
            continue
        if k in FC4_BYTES:                 # streaming W4: HBM-bound
            by = FC4_BYTES[k](B, S)
            out[k] = {"GBps": round(by / (us * 1e-6) / 1e9, 1), "bound": "hbm",
                      "frac": round(by / (us * 1e-6) / HBM_PEAK, 3)}
        elif k in fl:
            tf = fl[k] / (us * 1e-6) / 1e12
            out[k] = {"TFLOPs": round(tf, 2), "arith": KERNEL_ARITH.get(k, "f32"),
                      "peak": round(arith_peak(k) / 1e12, 1),
                      "frac": round(tf * 1e12 / arith_peak(k), 3)}
        elif k == "sample_gather":
            by = 2 * B * 4 * S * S * 5 + B * 24
            out[k] = {"GBps": round(by / (us * 1e-6) / 1e9, 1),
                      "frac": round(by / (us * 1e-6) / HBM_PEAK, 3)}
        elif k == "apply":
            by = 20 * P
            out[k] = {"GBps": round(by / (us * 1e-6) / 1e9, 1),
                      "frac": round(by / (us * 1e-6) / HBM_PEAK, 3)}
    return out


def acting_rate(net, cfg, S, iters=200, seed=5):
    """SURVEY 8(d) 'including acting' variant: per update one batch-1 greedy
    action (ddq_select_action on the newest state) and one synthetic-frame
    add_experience, then the fused training step (host-synchronous loop)."""
    from ddq.expgain import synthetic_transitions
    st, ac, rw, nt = synthetic_transitions(64, S, seed=seed)
    for i in range(5):
        net.select_action(st[i:i + 1])
        net.replay_add(int(ac[i]), int(rw[i]), st[i])
        net.step(cfg)
    net.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        j = i % 64
        net.select_action(st[j:j + 1])
        net.replay_add(int(ac[j]), int(rw[j]), st[j] if nt[j] else None)
        net.step(cfg)
    net.synchronize()
    dt = time.perf_counter() - t0
    return {"value": round(iters / dt, 2), "unit": "updates/s",
            "note": "eager step + batch-1 select_action + add_experience per update, "
                    "host-synchronous (%d updates)" % iters}


def dev_timer(net):
    """HIP-event timer on the ctx stream (torch events on an ExternalStream)."""
    import torch
    st = torch.cuda.ExternalStream(net.stream(), device=torch.device("cuda", net.device))

    def run(fn, iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / iters       # us per call
    return run


def gather_stress(S=64, N=1_000_000, sizes=(256, 4096, 32768), seed=3):
    """SURVEY 8(d) C5 gather stress: 1M-transition HBM ring (16.4 GB at 64x64),
    device draw + Caffe-layout gather of n transitions per launch.  Bytes per
    launch (algorithmic) = 2*n*4*S*S u8 read + 2*n*4*S*S*4 f32 write
    + n*(1+2+1) scalars read + n*(4+1+1)*4 written."""
    import ddq
    from ddq.expgain import synthetic_transitions
    net = ddq.DeepQNet(batch=32, frame=S)
    net.replay_create(N)
    st, ac, rw, nt = synthetic_transitions(4096, S, seed=seed)
    net.replay_fill_tiled(st, ac, rw, nt.astype(np.uint8), 12345, N)
    timer = dev_timer(net)
    out = []
    for n in sizes:
        bufs = net.batch_buffers(n)
        iters = max(5, min(200, (1 << 22) // n))
        net.replay_sample_batch(bufs, seed=seed)           # warm (allocates the bitmap)
        net.synchronize()
        us_all = timer(lambda: net.replay_sample_batch(bufs, seed=seed, check=False), iters)
        # gather alone over 16 pre-drawn index sets in rotation, so the slots
        # read are not still in the 256 MB Infinity Cache from the last call
        sets = []
        import torch
        for _ in range(16):
            net.replay_sample_batch(bufs, seed=seed)          # synchronises the ctx stream
            sets.append(bufs["idx"].clone())                  # on torch's current stream
        torch.cuda.synchronize()                              # clones done before the ctx reads them
        rot = [0]

        def gather_next():
            bufs["idx"] = sets[rot[0] % len(sets)]
            rot[0] += 1
            net.replay_gather_batch(bufs, check=False)
        us_g = timer(gather_next, iters)
        net._check(net.lib.ddq_replay_status(net.ctx))
        slot = 4 * S * S
        algo = 2 * n * slot * 5 + n * 4 + n * 24
        out.append({"n": n, "sample_gather_us": round(us_all, 2), "gather_us": round(us_g, 2),
                    "gather_GBps": round(algo / (us_g * 1e-6) / 1e9, 1),
                    "frac": round(algo / (us_g * 1e-6) / HBM_PEAK, 4),
                    "sample_gather_GBps": round(algo / (us_all * 1e-6) / 1e9, 1),
                    "algo_bytes": algo})
        del bufs
    net.close()
    return {"replay_slots": N, "frame": S, "bound": "hbm", "peak_GBps": HBM_PEAK / 1e9,
            "launches": out}


def frame_sweep(B=256, frames=range(16, 129, 8), steps=60, warmup=10, rule="rmsprop"):
    """batch 256, frame side 16..128 (results/cost-vs-image-size)."""
    import ddq
    from ddq.params import init_params_flat
    from ddq.expgain import synthetic_transitions
    res = []
    for S in frames:
        net = ddq.DeepQNet(batch=B, frame=S)
        theta = init_params_flat(S, seed=42)
        net.set_flat(0, theta)
        net.set_flat(1, theta)
        N = 30000
        net.replay_create(N)
        st, ac, rw, nt = synthetic_transitions(1024, S, seed=1)
        net.replay_fill_tiled(st, ac, rw, nt.astype(np.uint8), 0, N)
        cfg = net.step_cfg(rule, lr=1e-4, target_period=10, seed=1234)
        net.step_graph(cfg, warmup)
        net.synchronize()
        t0 = time.perf_counter()
        net.step_graph(cfg, steps)
        net.synchronize()
        dt = (time.perf_counter() - t0) / steps
        fl = net.step_flops()
        res.append({"frame": S, "updates_per_s": round(1 / dt, 2), "ms_per_step": round(dt * 1e3, 4),
                    "step_tflops": round(fl / dt / 1e12, 2),
                    "frac_of_f32_mfma_peak": round(fl / dt / F32_MFMA_PEAK, 4)})
        net.close()
    return {"batch": B, "config": "C3: deepq, batch 256, frame side S, rmsprop, 8-step graphs",
            "step_tflops_basis": "algorithmic f32 FLOPs of the whole step (SURVEY 8(d))",
            "f32_mfma_peak_TFLOPs": F32_MFMA_PEAK / 1e12, "frames": res}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--frame", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--replay", type=int, default=30000)
    ap.add_argument("--rule", default="rmsprop")
    ap.add_argument("--profile-steps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather-stress", action="store_true",
                    help="skip the C5 1M-slot gather stress (rank 0, N=1 only)")
    ap.add_argument("--chunks", type=int, default=20,
                    help="timed chunks for the step-time median/p10/p90 (0: skip)")
    ap.add_argument("--chunk-steps", type=int, default=24)
    ap.add_argument("--acting", action="store_true",
                    help="also time updates including acting (select_action + add_experience)")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C3 frame sweep")
    ap.add_argument("--sweep", action="store_true",
                    help="C3: also run the batch-256 frame-size sweep 16..128 (slow)")
    ap.add_argument("--eager", action="store_true", help="no hipGraph (debug)")
    ap.add_argument("--exchange", default="allreduce",
                    choices=["allreduce", "sharded", "server", "async"],
                    help="N>1 gradient exchange (include/ddq_hip.h enum ddq_exchange)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="allreduce: do not reduce the fc4 bucket under the conv backward")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="plain graph steps, each drawing + gathering its own minibatch at its "
                         "head (default: the next step's draw + gather ride on this step's "
                         "apply launch into a second minibatch buffer -- bit-identical results)")
    args = ap.parse_args()
    args.pipeline = not args.no_pipeline

    from ddq import dist as ddist
    rank, world, local = ddist.env_ranks()
    import torch
    dist = ddist.init_process_group(rank, world, "gloo")   # bootstrap only; data path is RCCL
    torch.cuda.set_device(local)

    import ddq
    B, S = args.batch, args.frame
    net = ddq.DeepQNet(batch=B, frame=S, device=local)
    from ddq.params import init_params_flat
    theta = init_params_flat(S, seed=42)            # identical on every rank
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    net.replay_create(args.replay)
    fill_replay(net, args.replay, S, seed=1000 + rank)
    if world > 1:
        ddist.setup_comm(net, rank, world)
    cfg = net.step_cfg(args.rule, lr=1e-4, target_period=10,
                       exchange=args.exchange if world > 1 else "none",
                       overlap=not args.no_overlap, seed=ddist.index_seed(1234, rank))

    def run(k):
        if args.eager:
            for _ in range(k):
                net.step(cfg)
        elif args.pipeline:
            net.step_pipelined(cfg, k)
        else:
            net.step_graph(cfg, k)

    # Step mode: capture every graph first (nothing launched), then agree on
    # the first mode every rank prepared (gloo MIN): a rank whose capture of the
    # comm-stream exchange is refused falls back TOGETHER with the others, so
    # no rank waits in an RCCL collective the rest abandoned.
    if args.eager:
        modes = [("eager", False)]
    elif args.pipeline:
        modes = [("pipelined", not args.no_overlap), ("graph", False), ("eager", False)]
    else:
        modes = [("graph", not args.no_overlap), ("graph", False), ("eager", False)]
    mode, ov = ddist.choose_step_mode(net, cfg, modes,
                                      log=lambda m: print("bench: " + m, file=sys.stderr))
    args.eager = mode == "eager"
    args.pipeline = mode == "pipelined"
    args.no_overlap = not ov
    run(args.warmup)
    net.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    net.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = ddist.max_over_ranks(time.perf_counter() - t0)
    loss = float(net.blob("loss"))

    # step-time distribution: chunks of graph steps bracketed by HIP events on
    # the ctx stream (no host sync inside a chunk)
    dist_ms = None
    if not args.eager and args.chunks > 0:
        timer = dev_timer(net)
        per = sorted(timer(lambda: run(args.chunk_steps), 1) / args.chunk_steps / 1e3
                     for _ in range(args.chunks))
        dist_ms = {"median": round(float(np.median(per)), 4),
                   "p10": round(float(np.percentile(per, 10)), 4),
                   "p90": round(float(np.percentile(per, 90)), 4),
                   "chunks": args.chunks, "steps_per_chunk": args.chunk_steps}

    # per-kernel device times (HIP events on the ctx stream), averaged
    prof = {}
    pcfg = cfg if args.exchange != "async" or world == 1 else \
        net.step_cfg(args.rule, lr=1e-4, target_period=10, exchange="none", seed=1234)
    for _ in range(args.profile_steps):
        for name, us in net.profile_step(pcfg):
            prof.setdefault(name, []).append(us)
    avg = {k: float(np.median(v)) for k, v in prof.items()}
    flops = kernel_flops(B, S)
    dom = max((k for k in avg if k in flops), key=lambda k: avg[k])
    # the roofline kernel's launch time: back-to-back launches between two
    # HIP events (the per-kernel events above add their own overhead)
    dom_us = net.time_layer(dom, 100) if dom.endswith("_fwd") and dom.startswith("conv") \
        else avg[dom]
    achieved = flops[dom] / (dom_us * 1e-6) / 1e12
    step_flops = net.step_flops()

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(world * args.steps / dt, 2),
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (random-policy Snake frames, Gaussian-init weights seed 42)",
            "config": {"workload": "deepq Snake DQN step, batch 32/GPU, 4-frame %dx%d, "
                                   "%d-slot HBM replay, %s apply, target sync every 10"
                                   % (S, S, args.replay, args.rule),
                       "global_batch": B * world, "frame": S,
                       "parallelism": "dp%d" % world, "graph": not args.eager,
                       "exchange": (args.exchange + ("" if args.no_overlap or
                                                     args.exchange != "allreduce"
                                                     else "+overlap")) if world > 1 else "none",
                       "pipelined": bool(args.pipeline and not args.eager)},
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3),
                         "peak": round(arith_peak(dom) / 1e12, 1), "unit": "TFLOP/s",
                         "frac": round(achieved * 1e12 / arith_peak(dom), 4),
                         "arith": KERNEL_ARITH.get(dom, "f32"),
                         "peak_basis": "algorithmic f32 FLOPs; peak = bf16 dense 2.5 PF/s over "
                                       "the bf16 products per f32 product (split: 6, split3: "
                                       "3; f32 MFMA: 157.3)",
                         "vs_f32_mfma_peak": round(achieved * 1e12 / F32_MFMA_PEAK, 4),
                         "traffic": pmc_traffic(dom, B, S), "traffic_unit": "bytes/launch",
                         "kernel_us": round(dom_us, 3),
                         "kernel_us_timing": "100 back-to-back launches between HIP events "
                                             "on the ctx stream",
                         "step_tflops": round(step_flops / (dt / args.steps) / 1e12, 3),
                         "step_frac": round(step_flops / (dt / args.steps) / F32_MFMA_PEAK, 4)},
            "kernels_us": {k: round(v, 2) for k, v in avg.items()},
            "kernel_roofline": kernel_roofline(avg, B, S, net.num_params),
            "step_ms_distribution": dist_ms,
            "final_loss": loss,
        }
        if args.acting and world == 1:
            out["with_acting"] = acting_rate(net, cfg, S)
        if not args.no_gather_stress and world == 1:
            out["gather_stress"] = gather_stress()
        if not args.no_sweep and world == 1:
            # C3 (BASELINE.json configs[2]): B = 256; the default line carries
            # the reduced sweep 16 / 64 / 128, --sweep the reference's 16..128/8
            out["frame_sweep"] = frame_sweep(frames=range(16, 129, 8) if args.sweep
                                             else (16, 64, 128))
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(B, S, seed=7)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    net.close()


if __name__ == "__main__":
    main()
