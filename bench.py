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
``roofline``: dominant kernel's in-step time (its own dispatch start / stop
events, hipExtLaunchKernel, in eager steps: ddq_profile_step) vs the peak of
the arithmetic it runs (split-bf16 kernels:
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
    # conv2_dgrad: conv2's data gradient with conv1's weight gradient fused
    # into its tiles (split.h w1_tile_wgrad): c2 split + c1 split3 FLOPs
    # deepq16's four launches (csrc/small.h, small_bwd.h): K1 tower_fwd (conv1..3
    # of both towers), K2 fc4_chain (fc4 forward of both towers, data and weight
    # gradients), K3 tower_bwd (conv3 / conv2 data gradients, conv1's weight
    # gradient), K4 wgrad_apply (conv2 / conv3 weight gradients)
    return {"conv1_fwd": 2 * c1, "conv2_fwd": 2 * c2, "conv3_fwd": 2 * c3, "fc4_fwd": 2 * fc,
            "fc4_bwd": fc, "conv3_dgrad": c3, "conv23_wgrad": c2 + c3, "conv2_dgrad": c2 + c1,
            "tower_fwd": 2 * (c1 + c2 + c3), "fc4_chain": 4 * fc, "tower_bwd": c3 + c2 + c1,
            "wgrad_apply": c2 + c3}


def kernel_parts(B, S):
    """(FLOPs, arithmetic) parts of each MFMA kernel: a fused kernel's ideal
    time is the sum of its parts at their arithmetic's peak."""
    s2, s3 = S // 2, S // 4
    c1 = 2.0 * B * S * S * 32 * 196
    c2 = 2.0 * B * s2 * s2 * 64 * 800
    c3 = 2.0 * B * s3 * s3 * 64 * 576
    return {"conv1_fwd": [(2 * c1, "split3")], "conv2_fwd": [(2 * c2, "split")],
            "conv3_fwd": [(2 * c3, "split")], "conv3_dgrad": [(c3, "split")],
            "conv23_wgrad": [(c2 + c3, "split")],
            "conv2_dgrad": [(c2, "split"), (c1, "split3")]}


def small_parts(B, S):
    """deepq16's fused launches: (FLOPs, arithmetic) parts (fc4 on the f32 MFMA)."""
    p = kernel_parts(B, S)
    fc = 2.0 * B * 512 * 64 * (S // 8) ** 2
    return {"tower_fwd": p["conv1_fwd"] + p["conv2_fwd"] + p["conv3_fwd"],
            "fc4_chain": [(4 * fc, "f32")],
            "tower_bwd": p["conv3_dgrad"] + p["conv2_dgrad"],
            "wgrad_apply": p["conv23_wgrad"]}


# rocprof kernel symbol (prefix) of each profiled step kernel
KERNEL_SYMBOL = {
    "sample_gather": "ddq::sample_gather_kernel",
    "conv1_fwd": "void ddq::split_conv1_kernel",
    "conv2_fwd": "void ddq::split_conv_kernel<32, 32, 64, 5,",
    "conv3_fwd": "void ddq::split_conv_kernel<64, 64, 64, 3, 8, 8, 2, 2,",
    "fc4_fwd": "void ddq::fc4_fwd_split_kernel",
    "head": "ddq::fc4_head_kernel",
    "fc4_bwd": "void ddq::fc4_bwd_kernel",
    "conv3_dgrad": "void ddq::split_conv_kernel<64, 64, 64, 3, 4, 8,",
    "conv23_wgrad": "void ddq::wgrads_pair_kernel",
    "conv2_dgrad": "void ddq::split_conv_kernel<64, 64, 32, 5,",
    "wgrad_reduce": "ddq::wgrad_reduce_kernel",
    "apply": "ddq::apply_kernel",
    "tower_fwd": "void ddq::sm16::tower_fwd16_kernel",
    "fc4_chain": "ddq::sm16::fc4_chain16_kernel",
    "tower_bwd": "void ddq::sm16::tower_bwd16_kernel",
    "wgrad_apply": "ddq::sm16::wgrad16_kernel",
}

# How each MFMA kernel computes its f32-exact result (csrc/split.h, wgrads.h):
# "split" = operands split into three bf16 planes, 6 bf16 products per f32
# product; "split3" = one operand exact in bf16 (the frames), 3 products;
# "f32" = v_mfma_f32_32x32x2_f32 / f32 VALU.  Its roofline peak is the bf16
# dense peak over the products per f32 product (the f32 MFMA peak for "f32").
KERNEL_ARITH = {
    "conv1_fwd": "split3", "conv2_fwd": "split", "conv3_fwd": "split", "conv23_wgrad": "split",
    "conv2_dgrad": "split+split3", "conv3_dgrad": "split", "fc4_fwd": "split", "fc4_bwd": "split",
    "tower_fwd": "split+split3", "tower_bwd": "split+split3", "wgrad_apply": "split",
    "fc4_chain": "f32",
}
BF16_MFMA_PEAK = 2.5e15       # MI355X_MICROARCH.md: dense bf16


def arith_peak(kernel, kind=None):
    kind = kind or KERNEL_ARITH.get(kernel, "f32")
    return {"split": BF16_MFMA_PEAK / 6, "split3": BF16_MFMA_PEAK / 3}.get(kind, F32_MFMA_PEAK)


def ideal_s(kernel, B, S):
    """Seconds of a kernel's FLOPs at the peaks of the arithmetic each part runs."""
    parts = kernel_parts(B, S)
    parts.update(small_parts(B, S))
    return sum(f / arith_peak(kernel, kind) for f, kind in parts[kernel])


def pmc_traffic(label, B, S):
    """(HBM bytes per launch of `label`, source file) from the newest committed
    step-only PMC summary (profiles/rNN_pmc_step.json: the bench's step chain
    alone, no exchange-path dispatches; tools/gpu/run.sh PMC=...: FETCH_SIZE x2
    + WRITE_SIZE, MI355X_MICROARCH.md gfx950 correction) -- a separate
    rocprofv3 --pmc run of the same bench command, NOT measured in this run;
    valid for the bench default shape only."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc_step.json")))
    if not paths:
        paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_pmc.json")))
    if (B, S) != (32, 64) or not paths:
        return None, None
    sym = KERNEL_SYMBOL.get(label)
    for name, e in json.load(open(paths[-1]))["kernels"].items():
        if sym and name.startswith(sym) and "hbm_bytes" in e:
            return round(e["hbm_bytes"]), os.path.relpath(paths[-1], ROOT)
    return None, None


def step_roofline(B, S, P):
    """Ideal time of one update step: every MFMA kernel at the peak of the
    arithmetic it runs (split: bf16 dense / 6, split3: / 3 -- csrc/split.h)
    plus the step's algorithmic HBM bytes at 8 TB/s (replay gather u8 read +
    f32 minibatch write, fc4 weights read by the two forwards and the data
    gradient, rmsprop apply 20 P).  The fraction measured / ideal is the
    step's roofline fraction (SURVEY 8(d) composite, split-aware)."""
    mfma_s = sum(ideal_s(k, B, S) for k in kernel_parts(B, S)) + \
        sum(kernel_flops(B, S)[k] / arith_peak(k) for k in ("fc4_fwd", "fc4_bwd"))
    K4 = 64 * (S // 8) ** 2
    gather = 2 * B * 4 * S * S + 2 * B * 4 * S * S * 4 + B * 24
    fc4 = 3 * 512 * K4 * 4
    apply_b = 20 * P
    hbm_s = (gather + fc4 + apply_b) / HBM_PEAK
    return {"ideal_us": round((mfma_s + hbm_s) * 1e6, 2), "mfma_us": round(mfma_s * 1e6, 2),
            "hbm_us": round(hbm_s * 1e6, 2), "hbm_bytes": gather + fc4 + apply_b}


def fill_replay(net, N, S, seed):
    from ddq.expgain import synthetic_transitions
    pool = min(N, 4096)
    st, ac, rw, nt = synthetic_transitions(pool, S, seed=seed)
    reps = (N + pool - 1) // pool
    net.replay_import(np.tile(st, (reps, 1, 1, 1))[:N], np.tile(ac, reps)[:N],
                      np.tile(rw, reps)[:N], np.tile(nt, reps)[:N].astype(np.uint8), 0, N)


def make_net(B, S, replay, device, rank):
    """The bench's worker: seed-42 Gaussian fillers (identical on every rank),
    a replay ring of `replay` synthetic Snake transitions (seed 1000 + rank)."""
    import ddq
    from ddq.params import init_params_flat
    net = ddq.DeepQNet(batch=B, frame=S, device=device)
    theta = init_params_flat(S, seed=42)
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    net.replay_create(replay)
    fill_replay(net, replay, S, seed=1000 + rank)
    return net


def preheat(B, S, local, ms):
    """Bring the chip to its running clocks before the measured context's W
    warmup steps: a THROWAWAY context (own weights, own max(1024, 4 B)-slot
    replay ring, exchange-free) runs pipelined step chains for `ms` wall milliseconds.
    The measured context's state is untouched.  Measured
    (tools/gpu/first_launch.py, profiles/r04_clock_ramp.txt): a chip idle
    for 10 ms runs the next 20 steps at 0.155-0.164 ms against 0.146 when
    busy, and 5 warmup steps (0.7 ms) do not bring it back."""
    if ms <= 0:
        return None
    ring = max(1024, 4 * B)                 # a ring the batch can draw from (B < valid)
    hot = make_net(B, S, ring, local, 0)
    cfg = hot.step_cfg("rmsprop", lr=1e-4, target_period=10, exchange="none", seed=99)
    hot.step_prepare(cfg, "pipelined")
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < ms / 1e3 and n < 100000:
        hot.step_pipelined(cfg, 24)
        hot.synchronize()
        n += 24
    return hot, {"ms": round((time.perf_counter() - t0) * 1e3, 1), "steps": n,
                 "work": "pipelined step chains of a throwaway context (own weights and "
                         "%d-slot replay, no exchange) before the W warmup steps; the "
                         "measured context is untouched" % ring}


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


PUBLISHED_CPU_MS = {16: 81.7, 32: 252.8, 64: 981.5, 128: 4044.0}   # results/cost-vs-image-size.txt


def cpu_baseline(B, S, seed, budget_s=12.0, max_steps=2000,
                 extra=((32, 16, 5.0), (256, 16, 5.0))):
    """Oracle C restatement (Caffe CPU algorithm: im2col + SGEMM, fp32, OpenMP)
    of the same update step, on all host cores and on one core (BASELINE.md
    section 2), with the reference's own published 2015 Caffe CPU time for
    context (results/cost-vs-image-size.txt:2-5, hardware unstated); `extra`
    (B, S, seconds): the same at deepq16 (the reference's headline, S = 16
    B = 32) and at a C3 sweep point (B = 256)."""
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
    published = PUBLISHED_CPU_MS.get(S)
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
    cfgs = []
    for eb, es, sec in extra:
        fl = lib.ddq_cpu_step_flops(eb, es)
        n, d = _cpu_updates(lib, eb, es, seed, cores, sec, max_steps)
        n1, d1 = _cpu_updates(lib, eb, es, seed, 1, sec / 2, max(2, max_steps // 8))
        e = {"batch": eb, "frame": es, "value": round(n / d, 4), "cores": cores,
             "gflops": round(fl * n / d / 1e9, 1), "sample": "%d updates, %.1f s" % (n, d),
             "single_core": {"value": round(n1 / d1, 4), "cores": 1,
                             "gflops": round(fl * n1 / d1 / 1e9, 1),
                             "sample": "%d updates, %.1f s" % (n1, d1)}}
        if eb == 32 and es in PUBLISHED_CPU_MS:
            e["reference_published"] = {"value": round(1000.0 / PUBLISHED_CPU_MS[es], 4),
                                        "unit": "updates/s (fwd+bwd only, Caffe CPU, "
                                                "%.1f ms)" % PUBLISHED_CPU_MS[es]}
        cfgs.append(e)
    out["configs"] = cfgs
    return out


def deepq16_line(steps=2000, warmup=100, rule="rmsprop"):
    """The reference's own headline shape, deepq16 (S = 16, B = 32,
    models/deepq/train_val.prototxt:8-11; results/cost-vs-image-size.txt:2):
    the same pipelined graph step on one GPU, 30 000-slot replay."""
    import ddq
    from ddq.params import init_params_flat
    B, S = 32, 16
    net = ddq.DeepQNet(batch=B, frame=S)
    theta = init_params_flat(S, seed=42)
    net.set_flat(0, theta)
    net.set_flat(1, theta)
    net.replay_create(30000)
    fill_replay(net, 30000, S, seed=1000)
    cfg = net.step_cfg(rule, lr=1e-4, target_period=10, seed=1234)
    net.step_prepare(cfg, "pipelined")
    net.step_pipelined(cfg, warmup)
    net.synchronize()
    t0 = time.perf_counter()
    net.step_pipelined(cfg, steps)
    net.synchronize()
    dt = (time.perf_counter() - t0) / steps
    rl = step_roofline(B, S, net.num_params)
    # the four launches' own dispatch times (eager steps, hipExtLaunchKernel
    # start / stop events on the ctx stream), median of 20, each against the
    # peak of the arithmetic it runs (kernel_roofline)
    prof = {}
    for _ in range(20):
        for name, us in net.profile_step(cfg):
            prof.setdefault(name, []).append(us)
    kus = {k: float(np.median(v)) for k, v in prof.items()}
    small_path = net.small_path()[0]
    net.close()
    return {"batch": B, "frame": S, "updates_per_s": round(1 / dt, 2),
            "ms_per_step": round(dt * 1e3, 4), "steps": steps, "small_path": small_path,
            "step_ideal_us": rl["ideal_us"], "step_frac": round(rl["ideal_us"] * 1e-6 / dt, 4),
            "kernels_us": {k: round(v, 2) for k, v in kus.items()},
            "kernel_roofline": kernel_roofline(kus, B, S, net.num_params),
            "reference_published_fwd_bwd_ms": PUBLISHED_CPU_MS[16]}


# algorithmic HBM bytes per launch of the fc4 kernels: W4 (512 x K fp32 per
# tower) plus activations in and out (K = 64 (S/8)^2)
FC4_BYTES = {
    "fc4_fwd": lambda B, S: 2 * (512 * 64 * (S // 8) ** 2 * 4 + B * 64 * (S // 8) ** 2 * 4),
    # the data gradient (the fused apply computes the weight gradient)
    "fc4_bwd": lambda B, S: 512 * 64 * (S // 8) ** 2 * 4 + B * 512 * 4 + B * 64 * (S // 8) ** 2 * 4,
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
                      "ideal_us": round(ideal_s(k, B, S) * 1e6, 3),
                      "frac": round(ideal_s(k, B, S) / (us * 1e-6), 3)}
            if "+" not in out[k]["arith"]:
                out[k]["peak"] = round(arith_peak(k) / 1e12, 1)
        elif k == "sample_gather":
            by = 2 * B * 4 * S * S * 5 + B * 24
            out[k] = {"GBps": round(by / (us * 1e-6) / 1e9, 1),
                      "frac": round(by / (us * 1e-6) / HBM_PEAK, 3)}
        elif k == "apply":
            # fused steps: every parameter is applied inside the slab-reduce
            # launch; this launch only carries the next step's draw + gather
            by = 2 * B * 4 * S * S * 5 + B * 24
            out[k] = {"GBps": round(by / (us * 1e-6) / 1e9, 1), "role": "prefetch gather",
                      "frac": round(by / (us * 1e-6) / HBM_PEAK, 3)}
        elif k == "wgrad_reduce":
            # slab reads + the fused rmsprop apply of every parameter (theta,
            # state read + written, gradient written: 20 P; fc4's x tile and
            # dh4 come from L2)
            by = slab_bytes(B, S) + 20 * P
            out[k] = {"GBps": round(by / (us * 1e-6) / 1e9, 1), "bound": "hbm",
                      "frac": round(by / (us * 1e-6) / HBM_PEAK, 3)}
    return out


def slab_bytes(B, S, target2=256, target3=256):
    """fp32 weight-gradient slab bytes per step (kernels.hip wgrad_splits_for /
    wgrads.h wgrads_groups at the product's group targets, csrc/common.h)."""
    def groups(rows, nts, target):
        g = max(1, target // nts)
        if g >= 16:
            g &= ~7
        g = max(1, min(g, rows))
        rpg = -(-rows // g)
        return -(-rows // rpg)
    band = 8
    while band > 1 and S % band:
        band //= 2
    np_ = lambda kc: -(-(kc + 1) // 64) * 64
    g1 = B * (S // band)
    g2 = groups(B * S // 2, 10, target2)
    g3 = groups(B * S // 4, 6, target3)
    return 4 * (g1 * 32 * np_(196) + g2 * 64 * np_(800) + g3 * 64 * np_(576))


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


EXCHANGE_PATHS = (   # (label, exchange, overlap, step mode)
    ("allreduce+overlap", "allreduce", True, "pipelined"),
    ("allreduce", "allreduce", False, "pipelined"),
    ("sharded", "sharded", False, "pipelined"),
    ("server", "server", False, "pipelined"),
    ("async", "async", False, "eager"),            # round-robin rounds, eager
    ("async-graph", "async", False, "graph"),      # round-robin rounds as hipGraphs
    ("async-ticket", "async", False, "ticket"))    # arrival order (AsyncTicketLoop)


def exchange_paths(net, rule, steps=240, warmup=24, profile=5):
    """The per-GPU path of BASELINE configs 4 / 5 measured on one GPU: every
    gradient exchange through a 1-rank RCCL communicator (the same kernels,
    RCCL calls, comm-stream overlap and graph capture as N > 1, without the
    wire time), against an exchange-free leg of the same length timed in this
    function (before and after the paths; their mean is the reference)."""
    import ddq
    from ddq import dist as ddist
    from ddq.params import init_params_flat
    out = {}
    base = net

    def free_leg():
        c0 = base.step_cfg(rule, lr=1e-4, target_period=10, exchange="none", seed=1234)
        base.step_prepare(c0, "pipelined")
        base.step_pipelined(c0, warmup)
        base.synchronize()
        t = 0.0
        for k in chunks:   # the same chunks (and drains) as the paths
            t0 = time.perf_counter()
            base.step_pipelined(c0, k)
            base.synchronize()
            t += time.perf_counter() - t0
        return steps / t
    # timed in 6 chunks (a drain between chunks): the total is the value, the
    # chunk median separates a host hiccup from the path's own cost (the
    # host-driven ticket leg varied 0.62 -- 0.79 across boxes)
    nch = 6   # (40-step chunks: whole 8-step pipelined and 10-round async graphs)
    chunks = [steps // nch + (1 if i < steps % nch else 0) for i in range(nch)]
    ref_before = free_leg()
    for label, ex, ov, mode in EXCHANGE_PATHS:
        if ex == "async":     # a fresh worker: once begun, a ctx runs async steps only
            net = ddq.DeepQNet(batch=base.batch, frame=base.frame, device=base.device)
            theta = init_params_flat(base.frame, seed=42)
            net.set_flat(0, theta)
            net.set_flat(1, theta)
            net.replay_create(30000)
            fill_replay(net, 30000, base.frame, seed=1000)
            ddist.setup_comm(net, 0, 1)
        else:
            net = base
            if "comm" not in out:
                ddist.setup_comm(net, 0, 1)
                out["comm"] = True
        cfg = net.step_cfg(rule, lr=1e-4, target_period=10, exchange=ex, overlap=ov, seed=1234)
        if mode != "ticket":
            net.step_prepare(cfg, mode)
        loop = ddist.AsyncTicketLoop(net, cfg, ddist.ticket_store(1), 0, 1) \
            if mode == "ticket" else None

        def run(k):
            if mode == "pipelined":
                net.step_pipelined(cfg, k)
            elif mode == "graph":
                net.step_graph(cfg, k)
            elif mode == "ticket":
                loop.run(k)
                net.synchronize()
            else:
                for _ in range(k):
                    net.step(cfg)
        run(warmup)
        net.synchronize()
        per = chunks
        ct = []
        for k in per:
            t0 = time.perf_counter()
            run(k)
            net.synchronize()
            ct.append(time.perf_counter() - t0)
        dt = sum(ct) / steps
        e = {"updates_per_s": round(1 / dt, 2), "ms_per_step": round(dt * 1e3, 4), "mode": mode,
             "chunk_median_updates_per_s": round(float(np.median([k / t for k, t in zip(per, ct)])), 2)}
        if ex != "async":
            prof = {}
            for _ in range(profile):
                for name, us in net.profile_step(cfg):
                    prof.setdefault(name, []).append(us)
            e["kernels_us"] = {k: round(float(np.median(v)), 2) for k, v in prof.items()}
        else:
            net.close()
        out[label] = e
    out.pop("comm", None)
    ref_after = free_leg()
    ref = 0.5 * (ref_before + ref_after)
    for e in out.values():
        e["vs_exchange_free"] = round(e["updates_per_s"] / ref, 4)
        e["chunk_median_vs_exchange_free"] = round(e["chunk_median_updates_per_s"] / ref, 4)
    return {"note": "world-1 RCCL communicator: the N>1 per-GPU step (kernels, RCCL calls, "
                    "comm-stream overlap, graphs) without wire time; vs_exchange_free = "
                    "this path's updates/s over an exchange-free pipelined leg of the same "
                    "length (%d steps after %d warmup, in the same 6 chunks) timed before and after the paths"
                    % (steps, warmup),
            "exchange_free": {"updates_per_s_before": round(ref_before, 2),
                              "updates_per_s_after": round(ref_after, 2)},
            "paths": out}


PUBLISHED_MESSAGING = {   # results/cost-vs-image-size.txt:2-5 (Caffe CPU worker, 2015)
    16: {"message_MB": 0.91, "generate_ms": 1.97, "load_ms": 0.93, "server_latency_ms": 5},
    32: {"message_MB": 2.49, "generate_ms": 4.18, "load_ms": 2.05, "server_latency_ms": 15},
    64: {"message_MB": 8.78, "generate_ms": 8.55, "load_ms": 5.11, "server_latency_ms": 40},
    128: {"message_MB": 33.94, "generate_ms": 27.47, "load_ms": 18.99, "server_latency_ms": 116}}


def messaging_costs(frames=(16, 32, 64, 128), B=32, trials=7):
    """The push/pull half the reference publishes (results/cost-vs-image-size
    .txt, results/server-latency.txt; harness barista/messaging.py:168-230 and
    the HTTP round trip of baristanet.py:105-123): per frame side, the gradient
    message through ddq/barista/messaging.py -- size, generate (device ->
    host copy of the gradient + framing) and load times, uncompressed and
    zlib -- and the HTTP round trips to a ddq.param_server.ParamServer (its
    model and apply on this GPU) on 127.0.0.1: POST /api/v1/update_model of
    that message (the reference's 'server latency') and GET
    /api/v1/latest_model.  Medians over `trials`."""
    import http.client
    import socket
    import threading
    import ddq
    from ddq.barista import messaging as M
    from ddq.param_server import ParamServer
    from ddq.params import init_params_flat

    def med(fn):
        ts = []
        for _ in range(trials):
            t0 = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3, r

    out = []
    for S in frames:
        net = ddq.DeepQNet(batch=B, frame=S)
        theta = init_params_flat(S, seed=42)
        net.set_flat(0, theta)
        net.set_flat(1, theta)
        net.replay_create(2048)
        fill_replay(net, 2048, S, seed=5)
        cfg = net.step_cfg("rmsprop", lr=1e-4, target_period=10, seed=1234)
        net.step(cfg)
        net.synchronize()
        e = {"frame": S, "params": int(net.num_params)}
        for comp in (False, True):
            gen_ms, msg = med(lambda: M.create_gradient_message(net, compress=comp))
            load_ms, _ = med(lambda: M.load_gradient_message(msg, compressed=comp))
            key = "zlib" if comp else "raw"
            e[key] = {"message_MB": round(len(msg) / 1e6, 4), "generate_ms": round(gen_ms, 3),
                      "load_ms": round(load_ms, 3)}
        raw = M.create_gradient_message(net)
        net.close()
        ps = ParamServer(frame=S, batch=B)
        ps.init_params(seed=42)
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        th = threading.Thread(target=ps.serve, kwargs={"port": port}, daemon=True)
        th.start()
        conn = None
        for _ in range(200):
            try:
                conn = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
                conn.request("GET", "/")
                conn.getresponse().read()
                break
            except OSError:
                conn = None
                time.sleep(0.01)

        def post():
            conn.request("POST", "/api/v1/update_model", body=raw,
                         headers={"Content-Type": "application/deepQ"})
            return conn.getresponse().read()

        def get():
            conn.request("GET", "/api/v1/latest_model",
                         headers={"Content-Type": "application/deepQ"})
            return conn.getresponse().read()
        post_ms, reply = med(post)
        get_ms, model = med(get)
        assert reply == b"Updated", reply
        e["server"] = {"update_roundtrip_ms": round(post_ms, 3),
                       "latest_model_roundtrip_ms": round(get_ms, 3),
                       "model_message_MB": round(len(model) / 1e6, 4)}
        conn.close()
        ps.shutdown()
        th.join(timeout=10)
        ps.net.close()
        if S in PUBLISHED_MESSAGING:
            e["reference_published"] = PUBLISHED_MESSAGING[S]
        out.append(e)
    return {"batch": B, "trials": trials,
            "note": "gradient message = the reference's framing + fp32 Q* payload "
                    "(ddq/barista/messaging.py); generate includes the device -> host copy "
                    "of the flat gradient; server round trips over HTTP/1.1 keep-alive on "
                    "127.0.0.1 to ParamServer (model + rmsprop apply on this GPU); "
                    "reference_published: results/cost-vs-image-size.txt (sys.getsizeof of "
                    "the message, Caffe CPU worker, 2015 hardware)",
            "frames": out}


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
        rl = step_roofline(B, S, net.num_params)
        res.append({"frame": S, "updates_per_s": round(1 / dt, 2), "ms_per_step": round(dt * 1e3, 4),
                    "step_tflops": round(fl / dt / 1e12, 2),
                    "frac_of_step_roofline": round(rl["ideal_us"] * 1e-6 / dt, 4),
                    "ideal_us": rl["ideal_us"],
                    "vs_f32_mfma_peak": round(fl / dt / F32_MFMA_PEAK, 4)})
        net.close()
    return {"batch": B, "config": "C3: deepq, batch 256, frame side S, rmsprop, 8-step graphs",
            "step_tflops_basis": "algorithmic f32 FLOPs of the whole step (SURVEY 8(d))",
            "frac_basis": "step_roofline(): each MFMA kernel at the peak of its arithmetic "
                          "(split / split3) + algorithmic HBM bytes at 8 TB/s",
            "f32_mfma_peak_TFLOPs": F32_MFMA_PEAK / 1e12, "frames": res}


def main():
    # the JSON line is the only thing on stdout: C-level writes to fd 1 (e.g.
    # RCCL's version banner at communicator init) go to stderr
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--frame", type=int, default=64)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--replay", type=int, default=30000)
    ap.add_argument("--rule", default="rmsprop")
    ap.add_argument("--profile-steps", type=int, default=20,
                    help="replays of the 8-step profiled graph (per-kernel in-step times)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather-stress", action="store_true",
                    help="skip the C5 1M-slot gather stress (rank 0, N=1 only)")
    ap.add_argument("--chunks", type=int, default=20,
                    help="timed chunks for the step-time median/p10/p90 (0: skip)")
    ap.add_argument("--chunk-steps", type=int, default=24)
    ap.add_argument("--acting", action="store_true",
                    help="also time updates including acting (select_action + add_experience)")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C3 frame sweep")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the dominant layer's isolated back-to-back timing (profiling runs)")
    ap.add_argument("--no-messaging", action="store_true",
                    help="skip the gradient-message / param-server round-trip costs (N=1)")
    ap.add_argument("--sweep", action="store_true",
                    help="C3: also run the batch-256 frame-size sweep 16..128 (slow)")
    ap.add_argument("--eager", action="store_true", help="no hipGraph (debug)")
    ap.add_argument("--preheat-ms", type=float, default=100.0,
                    help="wall ms of a throwaway context's step chains before the warmup "
                         "steps (the chip's clocks; 0: none)")
    ap.add_argument("--no-grad-store", action="store_true",
                    help="exchange-free steps do not store fc4's weight gradient "
                         "(DDQ_STEP_NO_GRAD_STORE; the update is unchanged)")
    ap.add_argument("--exchange", default="allreduce",
                    choices=["allreduce", "sharded", "server", "async"],
                    help="N>1 gradient exchange (include/ddq_hip.h enum ddq_exchange)")
    ap.add_argument("--force-exchange", default=None,
                    choices=["allreduce", "sharded", "server", "async"],
                    help="N=1: run this exchange through a 1-rank RCCL communicator (the N>1 "
                         "per-GPU path) for the main line")
    ap.add_argument("--no-exchange-paths", action="store_true",
                    help="skip the world-1 timing of every exchange path (N=1 only)")
    ap.add_argument("--async-order", default="rr", choices=["rr", "ticket"],
                    help="async exchange: round-robin rounds (deterministic) or arrival-order "
                         "tickets (ddq.dist.AsyncTicketLoop); a step = W pushes either way")
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

    B, S = args.batch, args.frame
    net = make_net(B, S, args.replay, local, rank)
    if world > 1:
        ddist.setup_comm(net, rank, world)
    elif args.force_exchange:
        ddist.setup_comm(net, 0, 1)
        args.exchange = args.force_exchange
    exchanged = world > 1 or bool(args.force_exchange)
    # --no-grad-store: exchange-free steps do not store fc4's weight gradient
    # (include/ddq_hip.h DDQ_STEP_NO_GRAD_STORE: the update is the same, bit
    # for bit, tests/test_gpu_parity.py)
    cfg = net.step_cfg(args.rule, lr=1e-4, target_period=10,
                       exchange=args.exchange if exchanged else "none",
                       overlap=not args.no_overlap, seed=ddist.index_seed(1234, rank),
                       store_grads=not args.no_grad_store)

    ticket = None
    if exchanged and args.exchange == "async" and args.async_order == "ticket":
        ticket = ddist.AsyncTicketLoop(net, cfg, ddist.ticket_store(world, rank), rank, world)

    def run(k):
        if ticket is not None:
            ticket.run(k * world)
        elif args.eager:
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
    if args.eager or ticket is not None:
        modes = [("eager", False)]
    elif exchanged and args.exchange == "async":
        modes = [("graph", False), ("eager", False)]
    elif args.pipeline:
        modes = [("pipelined", not args.no_overlap), ("graph", False), ("eager", False)]
    else:
        modes = [("graph", not args.no_overlap), ("graph", False), ("eager", False)]
    mode, ov = ddist.choose_step_mode(net, cfg, modes,
                                      log=lambda m: print("bench: " + m, file=sys.stderr))
    args.eager = mode == "eager"
    args.pipeline = mode == "pipelined"
    args.no_overlap = not ov
    # the same command without the preheat: W warmup steps, then 20 timed steps
    # on a chip fresh from idle (the measured context goes on from there)
    cold = None
    if args.preheat_ms > 0 and world == 1:
        run(args.warmup)
        net.synchronize()
        t0 = time.perf_counter()
        run(20)
        net.synchronize()
        cdt = time.perf_counter() - t0
        cold = {"value": round(20 / cdt, 2), "ms_per_step": round(cdt / 20 * 1e3, 4), "steps": 20,
                "warmup": args.warmup,
                "note": "W warmup + 20 timed steps before the preheat, chip fresh from idle "
                        "(clock ramp: profiles/r04_clock_ramp.txt)"}
    heated = preheat(B, S, local, args.preheat_ms)
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
    if heated is not None:
        heated[0].close()

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

    # per-kernel device times: eager steps whose every kernel carries start /
    # stop events of its own (hipExtLaunchKernel: the dispatch packet's
    # timestamps -- what rocprofv3's kernel trace reads -- with no marker
    # packets between the kernels), on the ctx stream the kernels run on;
    # median over --profile-steps steps
    pnet = net
    if exchanged and args.exchange == "async":   # an async ctx runs async steps only
        pnet = make_net(B, S, args.replay, local, rank)
    pcfg = cfg if not (exchanged and args.exchange == "async") else \
        pnet.step_cfg(args.rule, lr=1e-4, target_period=10, exchange="none", seed=1234,
                      store_grads=not args.no_grad_store)
    prof = {}
    for _ in range(max(1, args.profile_steps)):
        for name, us in pnet.profile_step(pcfg):
            prof.setdefault(name, []).append(us)
    avg = {k: float(np.median(v)) for k, v in prof.items()}
    flops = kernel_flops(B, S)
    dom = max((k for k in avg if k in flops), key=lambda k: avg[k])
    dom_us = avg[dom]
    # for reference: the same layer launched 100 times back to back on the same
    # cache-warm input (not the roofline figure)
    iso_us = pnet.time_layer(dom, 100) if dom.endswith("_fwd") and dom.startswith("conv") \
        and not args.no_isolated else None
    if pnet is not net:
        pnet.close()
    achieved = flops[dom] / (dom_us * 1e-6) / 1e12
    # peak of the arithmetic the kernel runs (a fused kernel: its FLOPs over
    # the ideal time of its parts)
    dom_peak = flops[dom] / ideal_s(dom, B, S)
    step_flops = net.step_flops()
    step_rl = step_roofline(B, S, net.num_params)
    traffic, traffic_src = pmc_traffic(dom, B, S)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(world * args.steps / dt, 2),
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "preheat": heated[1] if heated is not None else None,
            "no_preheat_20": cold,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (random-policy Snake frames, Gaussian-init weights seed 42)",
            "config": {"workload": "deepq Snake DQN step, batch 32/GPU, 4-frame %dx%d, "
                                   "%d-slot HBM replay, %s apply, target sync every 10"
                                   % (S, S, args.replay, args.rule),
                       "preheat_ms": args.preheat_ms,
                       "global_batch": B * world, "frame": S,
                       "parallelism": "dp%d" % world, "graph": not args.eager,
                       "exchange": (args.exchange + ("" if args.no_overlap or
                                                     args.exchange != "allreduce"
                                                     else "+overlap")) if exchanged else "none",
                       "pipelined": bool(args.pipeline and not args.eager),
                       "grad_store": "fc4 weight gradient stored" if not args.no_grad_store or exchanged
                                     else "fc4 weight gradient applied, not stored "
                                          "(DDQ_STEP_NO_GRAD_STORE)"},
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3),
                         "peak": round(dom_peak / 1e12, 1), "unit": "TFLOP/s",
                         "frac": round(achieved * 1e12 / dom_peak, 4),
                         "arith": KERNEL_ARITH.get(dom, "f32"),
                         "peak_basis": "algorithmic f32 FLOPs; peak = bf16 dense 2.5 PF/s over "
                                       "the bf16 products per f32 product (split: 6, split3: "
                                       "3; f32 MFMA: 157.3)",
                         "vs_f32_mfma_peak": round(achieved * 1e12 / F32_MFMA_PEAK, 4),
                         "traffic": traffic, "traffic_unit": "bytes/launch",
                         "traffic_source": traffic_src,
                         "kernel_us": round(dom_us, 3),
                         "kernel_us_timing": "in-step: median over %d eager steps of the "
                                             "kernel's own dispatch start / stop "
                                             "(hipExtLaunchKernel events on the ctx stream)"
                                             % max(1, args.profile_steps),
                         "isolated_us": None if iso_us is None else round(iso_us, 3),
                         "isolated_timing": "the same layer, 100 back-to-back launches on one "
                                            "cache-warm input (not the roofline figure)",
                         "step_tflops": round(step_flops / (dt / args.steps) / 1e12, 3),
                         "step_ideal_us": step_rl["ideal_us"],
                         "step_frac": round(step_rl["ideal_us"] * 1e-3 / (dt / args.steps * 1e3), 4),
                         "step_frac_basis": "step_roofline(): MFMA kernels at their "
                                            "arithmetic's peak + algorithmic HBM bytes"},
            "kernels_us": {k: round(v, 2) for k, v in avg.items()},
            "kernels_us_timing": "each kernel's own dispatch start / stop in eager steps "
                                 "(ddq_profile_step, hipExtLaunchKernel events); compare "
                                 "profiles/rNN_kernel_stats_step.csv (rocprofv3, graph replay)",
            "kernel_roofline": kernel_roofline(avg, B, S, net.num_params),
            "step_ms_distribution": dist_ms,
            "final_loss": loss,
        }
        if args.acting and world == 1:
            out["with_acting"] = acting_rate(net, cfg, S)
        if not args.no_gather_stress and world == 1:
            out["gather_stress"] = gather_stress()
        if not args.no_sweep and world == 1:
            out["deepq16"] = deepq16_line()
            # C3 (BASELINE.json configs[2]): B = 256; the default line carries
            # the reduced sweep 16 / 64 / 128, --sweep the reference's 16..128/8
            out["frame_sweep"] = frame_sweep(frames=range(16, 129, 8) if args.sweep
                                             else (16, 64, 128))
        if not args.no_messaging and world == 1:
            out["messaging"] = messaging_costs()
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(B, S, seed=7)
        if not args.no_exchange_paths and world == 1 and not args.force_exchange:
            out["exchange_paths"] = exchange_paths(net, args.rule)
        print(json.dumps(out), file=json_out, flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    net.close()


if __name__ == "__main__":
    main()
