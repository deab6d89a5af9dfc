"""Two shard engines in one process (exchange summed on the device with torch)
against one engine over all samples, several consecutive steps."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from quadrotor_manipulator_mppi_amd.engine import Engine, make_config
model = sys.argv[1] if len(sys.argv) > 1 else "arm"
K, H = 2048, 32
state = np.array([0, 0, 1, 0, 0, 0, 1] + [1.57, 1.7, 0, 4.4, 0, 4.71, 0.0] + [0.0] * 7, np.float64)
tgt = ([0.1029, 0.4055, 1.6498], [-0.5, -0.5, 0.5, -0.5])
full = Engine(make_config(model, n_samples=2 * K, n_horizon=H, seed=5))
full.set_target(*tgt)
shards = [Engine(make_config(model, n_samples=K, n_horizon=H, seed=5, shard_rank=r, shard_count=2)) for r in range(2)]
slot = shards[0].exchange_slot_floats()
bufs = [torch.zeros(2 * slot, device="cuda") for _ in range(2)]
for sh, b in zip(shards, bufs):
    sh.set_target(*tgt)
    sh.bind_exchange(b.data_ptr())
for step in range(6):
    out_f, u0_f, st_f = full.step(state)
    for sh in shards:
        sh.set_state(state)
        sh.rollout()
        sh.synchronize()
    total = bufs[0] + bufs[1]
    torch.cuda.synchronize()
    hdr = [b.view(2, -1)[:, :4].cpu().numpy() for b in bufs]
    for sh, b in zip(shards, bufs):
        b.copy_(total)
        torch.cuda.synchronize()
        sh.finalize()
    outs = [sh.read_outputs() for sh in shards]
    print(f"step {step}: full u0 {u0_f[0][:3]}  shard0 u0 {outs[0][1][0][:3]} shard1 u0 {outs[1][1][0][:3]}")
    print("   slot headers rank0-buf:", hdr[0].tolist(), " rank1-buf:", hdr[1].tolist())
    print("   finite:", np.isfinite(outs[0][0]).all(), np.isfinite(outs[1][0]).all(), "max|du0|", np.abs(outs[0][1] - u0_f).max())
