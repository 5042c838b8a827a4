"""Per-kernel device times of the training step at a few frame sizes (the C3
sweep's edge-tile frames beside exact ones): python tools/frame_kernels.py
[B] [S ...].  Prints one JSON line per frame: step time (8-step graphs) and
the median per-kernel event times of profile_step (eager, HIP events)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "distributed-deep-q_amd"))


def main():
    import ddq
    from ddq.params import init_params_flat
    from ddq.expgain import synthetic_transitions
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    frames = [int(s) for s in sys.argv[2:]] or [32, 40, 64, 72, 104]
    for S in frames:
        net = ddq.DeepQNet(batch=B, frame=S)
        theta = init_params_flat(S, seed=42)
        net.set_flat(0, theta)
        net.set_flat(1, theta)
        N = 30000
        net.replay_create(N)
        st, ac, rw, nt = synthetic_transitions(1024, S, seed=1)
        net.replay_fill_tiled(st, ac, rw, nt.astype(np.uint8), 0, N)
        cfg = net.step_cfg("rmsprop", lr=1e-4, target_period=10, seed=1234)
        net.step_graph(cfg, 16)
        net.synchronize()
        t0 = time.perf_counter()
        net.step_graph(cfg, 64)
        net.synchronize()
        dt = (time.perf_counter() - t0) / 64
        prof = {}
        for _ in range(5):
            for name, us in net.profile_step(cfg):
                prof.setdefault(name, []).append(us)
        k = {n: round(float(np.median(v)), 1) for n, v in prof.items()}
        print(json.dumps({"B": B, "S": S, "updates_per_s": round(1 / dt, 1),
                          "ms_per_step": round(dt * 1e3, 4), "kernels_us": k}), flush=True)
        net.close()


if __name__ == "__main__":
    main()
