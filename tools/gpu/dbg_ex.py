import sys, numpy as np
sys.path[:0]=['.', 'distributed-deep-q_amd']
import ddq
from oracle import ref_numpy as ref
sys.path.insert(0, 'tests')
from test_gpu_exchange import make_group
W,S=3,16
nets, arr, theta = make_group(ddq, ref, W, S)
for step in range(3):
    cfg = nets[0].step_cfg("rmsprop", lr=1e-3, target_period=0, exchange="server", seed=40+step)
    ddq.DeepQNet.group_step(nets, cfg, arr)
    for r, n in enumerate(nets):
        g = n.get_grads_flat(); t = n.get_flat(0); o = n.optimizer_state(); p = n.get_flat(1)
        bad = np.where(np.isnan(g))[0]
        print(step, r, "grad nan", bad.size, bad[:5], "theta nan", np.isnan(t).sum(), "opt nan", np.isnan(o).sum(),
              "loss", n.blob("loss"), "Qout nan", np.isnan(n.blob("Q_out")).sum(), "P nan", np.isnan(p).sum(), "opt min", np.nanmin(o))
