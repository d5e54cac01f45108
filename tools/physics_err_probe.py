"""GPU probe: physics error of the HIP kernel and of the float32 oracle against the float64 oracle
(one env step = 4 substeps from randomised states, 64 envs), per quantity - the data the derived
tolerances of tests/test_gpu_parity.py are set from.  Prints one JSON line per (task, seed)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from oracle_backend import make_env, simulate64  # noqa: E402
from test_gpu_parity import randomize_state, sync  # noqa: E402

QTY = {"root_pose": lambda e: e.root_states[:, :7], "root_vel": lambda e: e.root_states[:, 7:],
       "dof_pos": lambda e: e.dof_pos, "dof_vel": lambda e: e.dof_vel, "torques": lambda e: e.torques,
       "contact_forces": lambda e: e.contact_forces}

for task in sys.argv[1:] or ["go1_flat_bench", "go1_rough", "anymal_c_rough"]:
    ora = make_env(task, num_envs=64, device="cpu", backend="oracle")
    dev = make_env(task, num_envs=64, device="cuda:0", backend="lgx")
    for seed in range(8):
        gen = torch.Generator().manual_seed(seed)
        randomize_state(ora, gen, standing=seed % 2 == 0)
        sync(ora, dev)
        if hasattr(dev, "terrain_types"):
            dev.terrain_types.copy_(ora.terrain_types)
        s0 = {k: getattr(ora, k).clone() for k in ("root_states", "dof_state", "torques", "_contact_forces_full")}
        simulate64(ora, 4)
        t64 = {k: f(ora).clone().double() for k, f in QTY.items()}
        for k, v in s0.items():
            getattr(ora, k).copy_(v)
        ora.simulate(4)
        dev.simulate(4)
        torch.cuda.synchronize()
        row = {"task": task, "seed": seed}
        for k, f in QTY.items():
            eh = (f(dev).cpu().double() - t64[k]).abs()
            eo = (f(ora).double() - t64[k]).abs()
            row[k] = {"hip": eh.max().item(), "f32": eo.max().item(), "hip_env_max": eh.view(64, -1).max(1).values.topk(3).values.tolist(),
                      "f32_env_max": eo.view(64, -1).max(1).values.topk(3).values.tolist(), "scale": t64[k].abs().max().item()}
        print(json.dumps(row), flush=True)
