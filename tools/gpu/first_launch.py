"""Where the driver's short timed region (--steps 20 --warmup 5) loses time
against the steady-state chunks: host-timed chains on fresh contexts, with the
timed chain's graphs launched before or not, an idle gap before it, and the
cost of the bracketing synchronisation alone."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "distributed-deep-q_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def fresh():
    net = bench.make_net(32, 64, 30000, 0, 0)
    cfg = net.step_cfg("rmsprop", lr=1e-4, target_period=10, exchange="none",
                       overlap=True, seed=1234)
    net.step_prepare(cfg, "pipelined")
    return net, cfg


def timed(net, cfg, k):
    net.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    net.step_pipelined(cfg, k)
    net.synchronize()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


def case(name, warm, k=20, gap=0.0, repeat=1):
    net, cfg = fresh()
    for w in warm:
        net.step_pipelined(cfg, w)
    net.synchronize()
    if gap:
        time.sleep(gap)
    ms = [timed(net, cfg, k) for _ in range(repeat)]
    print(f"{name:40s} " + " ".join(f"{m:.4f}" for m in ms), flush=True)


def preheat_cases():
    for reps in (0, 400, 1200, 4000, 12000):
        net, cfg = fresh()
        t0 = time.perf_counter()
        if reps:
            net.time_layer("conv2_fwd", reps)
        ph = (time.perf_counter() - t0) * 1e3
        net.step_pipelined(cfg, 5)
        ms = timed(net, cfg, 20)
        print(f"preheat conv2_fwd x{reps:5d} ({ph:6.1f} ms), warm 5, time 20: {ms:.4f}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "preheat":
        return preheat_cases()
    net, cfg = fresh()
    net.step_pipelined(cfg, 5)
    net.synchronize()
    ts = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        net.synchronize()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    print(f"sync pair alone (us): min {min(ts):.1f} median {sorted(ts)[10]:.1f}", flush=True)
    case("warm 5, time 20 x4 (driver)", [5], repeat=4)
    case("warm 5,20 (same graphs), time 20", [5, 20])
    case("warm 20, time 20", [20])
    case("warm 5, gap 0.1 s, time 20", [5], gap=0.1)
    case("warm 5, time 24 x3", [5], k=24, repeat=3)
    case("warm 50, time 500", [50], k=500)
    net, cfg = fresh()
    net.step_pipelined(cfg, 500)
    net.synchronize()
    timer = bench.dev_timer(net)
    for k in (20, 24):
        host, dev, call = [], [], []
        for _ in range(8):
            net.synchronize()
            t0 = time.perf_counter()
            net.step_pipelined(cfg, k)
            t1 = time.perf_counter()
            net.synchronize()
            host.append((time.perf_counter() - t0) / k * 1e3)
            call.append((t1 - t0) * 1e6)
        for _ in range(8):
            dev.append(timer(lambda: net.step_pipelined(cfg, k), 1) / k / 1e3)
        print(f"after 500 warm, k={k}: host ms/step {' '.join(f'{x:.4f}' for x in host)}", flush=True)
        print(f"  host call us {' '.join(f'{x:.0f}' for x in call)}", flush=True)
        print(f"  device-event ms/step {' '.join(f'{x:.4f}' for x in dev)}", flush=True)
    for gap in (0.01, 0.1, 1.0):
        time.sleep(gap)
        d = timer(lambda: net.step_pipelined(cfg, 20), 1) / 20 / 1e3
        print(f"after idle {gap} s: device-event ms/step (20) {d:.4f}", flush=True)


if __name__ == "__main__":
    main()
