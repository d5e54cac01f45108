"""GPU probe: physics error of the HIP kernel and of the float32 oracle against the float64 oracle
(one env step = 4 substeps from randomised states, 64 envs), per quantity - the data the derived
tolerances of tests/test_gpu_parity.py are set from - and, for every env above the worst-env
bound, the near-threshold branch flip that explains it (test_gpu_parity.explain_outliers: the
decision, its substep and relative margin, HIP's error before and on the flipped branch).
Prints one JSON line per (task, seed).  Usage: python tools/physics_err_probe.py [tasks...]
[--seeds N]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_gpu_parity as P  # noqa: E402
from oracle_backend import make_env  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
nseeds = int(sys.argv[sys.argv.index("--seeds") + 1]) if "--seeds" in sys.argv else 8
if "--seeds" in sys.argv:
    args.remove(sys.argv[sys.argv.index("--seeds") + 1])
for task in args or ["go1_flat_bench", "go1_rough", "anymal_c_rough"]:
    ora = make_env(task, num_envs=64, device="cpu", backend="oracle")
    dev = make_env(task, num_envs=64, device="cuda:0", backend="lgx")
    for seed in list(range(nseeds)) + ([100, 101, 102] if "rough" in task else []):
        gen = torch.Generator().manual_seed(seed)
        # (seeds 100-102: the states of test_physics_rough_terrain_derived_tolerance)
        P.randomize_state(ora, gen, standing=(seed != 101) if seed >= 100 else seed % 2 == 0)
        P.sync(ora, dev)
        if hasattr(dev, "terrain_types"):
            dev.terrain_types.copy_(ora.terrain_types)
        t64 = P.float64_truth(ora, 4)
        ora.simulate(4)
        dev.simulate(4)
        torch.cuda.synchronize()
        row = {"task": task, "seed": seed}
        for k, f in P.PHYS_QTY.items():
            eh = (f(dev).cpu().double() - t64[k]).abs()
            eo = (f(ora).double() - t64[k]).abs()
            row[k] = {"hip": eh.max().item(), "f32": eo.max().item(),
                      "hip_env_max": eh.view(64, -1).max(1).values.topk(3).values.tolist(),
                      "f32_env_max": eo.view(64, -1).max(1).values.topk(3).values.tolist(),
                      "scale": t64[k].abs().max().item()}
        n0 = len(P.BRANCH_FLIPS)
        try:
            P.check_derived(t64, {k: f(ora) for k, f in P.PHYS_QTY.items()}, {k: f(dev) for k, f in P.PHYS_QTY.items()})
            row["check"] = "pass"
        except AssertionError as e:
            row["check"] = "FAIL: " + str(e)[:600]
        row["explained_outliers"] = P.BRANCH_FLIPS[n0:]
        print(json.dumps(row), flush=True)
