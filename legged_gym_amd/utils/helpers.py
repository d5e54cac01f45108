"""Config / CLI / seeding / checkpoint-path helpers of the drop-in boundary.

Behaviour follows legged_gym/utils/helpers.py (cited per function).  The Isaac Gym pieces
(`gymapi.SimParams`, `gymutil.parse_arguments`) are replaced by `SimParams` and an argparse
parser accepting the same flags.
"""
import argparse
import copy
import os
import random

import numpy as np

from legged_gym_amd import LEGGED_GYM_ROOT_DIR  # noqa: F401


def class_to_dict(obj) -> dict:
    """helpers.py:41-56 — recursive, keys in `dir()` order (alphabetical), private names skipped."""
    if not hasattr(obj, "__dict__"):
        return obj
    out = {}
    for key in dir(obj):
        if key.startswith("_"):
            continue
        val = getattr(obj, key)
        if isinstance(val, list):
            out[key] = [class_to_dict(v) for v in val]
        else:
            out[key] = class_to_dict(val)
    return out


def update_class_from_dict(obj, d):
    """helpers.py:58-65."""
    for key, val in d.items():
        attr = getattr(obj, key, None)
        if isinstance(attr, type):
            update_class_from_dict(attr, val)
        else:
            setattr(obj, key, val)


def set_seed(seed):
    """helpers.py:67-77 (seed == -1 draws a random seed)."""
    import torch
    if seed == -1:
        seed = np.random.randint(0, 10000)
    print(f"Setting seed: {seed}")
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    return seed


class SimParams:
    """Stand-in for gymapi.SimParams: the fields the lgx backend consumes.

    dt is stored as a float32 value (PhysX keeps it as a C float), which is why the
    reference ends up with dt = 4 * 0.004999999888 and max_episode_length = 1001
    (legged_robot.py:770-777)."""

    def __init__(self):
        self.dt = float(np.float32(1.0 / 60.0))
        self.substeps = 1
        self.gravity = [0.0, 0.0, -9.81]
        self.up_axis = 1
        self.use_gpu_pipeline = True
        self.physx = argparse.Namespace(num_threads=10, solver_type=1, num_position_iterations=4,
                                        num_velocity_iterations=0, contact_offset=0.01, rest_offset=0.0,
                                        bounce_threshold_velocity=0.5, max_depenetration_velocity=1.0,
                                        max_gpu_contact_pairs=2 ** 23, default_buffer_size_multiplier=5,
                                        contact_collection=2, use_gpu=True, num_subscenes=0)
        self.lgx = None


def parse_sim_params(args, cfg):
    """helpers.py:79-101: SimParams from CLI args, overridden by the cfg's "sim" dict."""
    sp = SimParams()
    sp.use_gpu_pipeline = getattr(args, "use_gpu_pipeline", True)
    sp.physx.use_gpu = getattr(args, "use_gpu", True)
    sp.physx.num_subscenes = getattr(args, "subscenes", 0)
    if "sim" in cfg:
        s = cfg["sim"]
        for k, v in s.items():
            if k == "physx":
                for pk, pv in v.items():
                    setattr(sp.physx, pk, pv)
            elif k == "dt":
                sp.dt = float(np.float32(v))
            else:
                setattr(sp, k, v)
    if getattr(args, "num_threads", 0) > 0:
        sp.physx.num_threads = args.num_threads
    return sp


def get_load_path(root, load_run=-1, checkpoint=-1):
    """helpers.py:103-125: last run (lexicographic) and last model (zero-padded sort)."""
    try:
        runs = sorted(os.listdir(root))
        if "exported" in runs:
            runs.remove("exported")
        last_run = os.path.join(root, runs[-1])
    except Exception as e:
        raise ValueError("No runs in this directory: " + root) from e
    load_run = last_run if load_run == -1 else os.path.join(root, load_run)
    if checkpoint == -1:
        models = [f for f in os.listdir(load_run) if "model" in f]
        models.sort(key=lambda m: "{0:0>15}".format(m))
        model = models[-1]
    else:
        model = f"model_{checkpoint}.pt"
    return os.path.join(load_run, model)


def update_cfg_from_args(env_cfg, cfg_train, args):
    """helpers.py:127-150."""
    if env_cfg is not None and getattr(args, "num_envs", None) is not None:
        env_cfg.env.num_envs = args.num_envs
    if cfg_train is not None:
        for name, target in (("seed", None), ("max_iterations", "max_iterations"), ("experiment_name", "experiment_name"),
                             ("run_name", "run_name"), ("load_run", "load_run"), ("checkpoint", "checkpoint")):
            val = getattr(args, name, None)
            if val is None:
                continue
            if target is None:
                cfg_train.seed = val
            else:
                setattr(cfg_train.runner, target, val)
        if getattr(args, "resume", False):
            cfg_train.runner.resume = True
    return env_cfg, cfg_train


def get_args(argv=None):
    """helpers.py:152-178 plus the gymutil flags the reference relies on."""
    p = argparse.ArgumentParser(description="RL Policy")
    p.add_argument("--task", type=str, default="anymal_c_flat")
    p.add_argument("--resume", action="store_true", default=False)
    p.add_argument("--experiment_name", type=str)
    p.add_argument("--run_name", type=str)
    p.add_argument("--load_run", type=str)
    p.add_argument("--checkpoint", type=int)
    p.add_argument("--headless", action="store_true", default=False)
    p.add_argument("--horovod", action="store_true", default=False)   # inert, as in the reference
    p.add_argument("--rl_device", type=str, default="cuda:0")
    p.add_argument("--num_envs", type=int)
    p.add_argument("--seed", type=int)
    p.add_argument("--max_iterations", type=int)
    # gymutil.parse_arguments flags
    p.add_argument("--sim_device", type=str, default="cuda:0")
    p.add_argument("--pipeline", type=str, default="gpu")
    p.add_argument("--graphics_device_id", type=int, default=0)
    p.add_argument("--num_threads", type=int, default=0)
    p.add_argument("--subscenes", type=int, default=0)
    p.add_argument("--physx", action="store_true", default=True)
    p.add_argument("--flex", action="store_true", default=False)
    args = p.parse_args(argv)
    dev = args.sim_device
    args.sim_device_type = dev.split(":")[0]
    args.compute_device_id = int(dev.split(":")[1]) if ":" in dev else 0
    args.use_gpu_pipeline = args.pipeline in ("gpu", "cuda")
    args.use_gpu = args.sim_device_type == "cuda"
    args.physics_engine = 0
    args.sim_device_id = args.compute_device_id
    args.sim_device = args.sim_device_type + (f":{args.sim_device_id}" if args.sim_device_type == "cuda" else "")
    return args


def _plain_actor(actor):
    """The actor MLP rebuilt from plain nn.Linear layers on the CPU (no dependency on this package
    in the exported module)."""
    import torch
    import torch.nn as nn
    layers = []
    for m in actor:
        if isinstance(m, nn.Linear):
            lin = nn.Linear(m.in_features, m.out_features)
            with torch.no_grad():
                lin.weight.copy_(m.weight.detach().cpu())
                lin.bias.copy_(m.bias.detach().cpu())
            layers.append(lin)
        else:
            layers.append(copy.deepcopy(m).to("cpu"))
    return nn.Sequential(*layers)


def export_policy_as_jit(actor_critic, path):
    """helpers.py:180-190: TorchScript export of the actor MLP as policy_1.pt, or, for a recurrent
    policy (one with `memory_a`), of memory + actor as policy_lstm_1.pt (PolicyExporterLSTM)."""
    import torch
    if hasattr(actor_critic, "memory_a"):
        PolicyExporterLSTM(actor_critic).export(path)
        return
    os.makedirs(path, exist_ok=True)
    torch.jit.script(_plain_actor(actor_critic.actor)).save(os.path.join(path, "policy_1.pt"))


def _policy_exporter_lstm_cls():
    import torch

    class PolicyExporterLSTM(torch.nn.Module):
        """helpers.py:193-219: the actor's LSTM + MLP as one TorchScript module that carries its
        (layers, 1, hidden) h / c state across calls; reset_memory() zeroes it."""

        def __init__(self, actor_critic):
            super().__init__()
            self.actor = _plain_actor(actor_critic.actor)
            self.is_recurrent = actor_critic.is_recurrent
            self.memory = copy.deepcopy(actor_critic.memory_a.rnn).cpu()
            self.register_buffer("hidden_state", torch.zeros(self.memory.num_layers, 1, self.memory.hidden_size))
            self.register_buffer("cell_state", torch.zeros(self.memory.num_layers, 1, self.memory.hidden_size))

        def forward(self, x):
            out, (h, c) = self.memory(x.unsqueeze(0), (self.hidden_state, self.cell_state))
            self.hidden_state[:] = h
            self.cell_state[:] = c
            return self.actor(out.squeeze(0))

        @torch.jit.export
        def reset_memory(self):
            self.hidden_state[:] = 0.
            self.cell_state[:] = 0.

        def export(self, path):
            os.makedirs(path, exist_ok=True)
            self.to("cpu")
            torch.jit.script(self).save(os.path.join(path, "policy_lstm_1.pt"))

    return PolicyExporterLSTM


def PolicyExporterLSTM(actor_critic):  # noqa: N802  (the reference's class name; torch imported lazily)
    return _policy_exporter_lstm_cls()(actor_critic)


