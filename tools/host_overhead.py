"""Host-side cost of the rollout loop vs its GPU time (go1_rough, 4096 envs): is collection
launch-bound?  Prints per-step host time of act + env.step + process_env_step (no sync inside)
and the synchronized wall time per step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import legged_gym_amd.envs  # noqa: E402,F401
from legged_gym_amd.utils.helpers import get_args  # noqa: E402
from legged_gym_amd.utils.task_registry import task_registry  # noqa: E402

task = "go1_rough"
env_cfg, train_cfg = task_registry.get_cfgs(task)
env_cfg.env.num_envs = 4096
cli = get_args(["--sim_device", "cuda:0", "--rl_device", "cuda:0", "--headless", "--task", task])
env, _ = task_registry.make_env(task, args=cli, env_cfg=env_cfg)
runner, _ = task_registry.make_alg_runner(env, name=task, args=cli, train_cfg=train_cfg, log_root=None)
runner.learn(2)
alg = runner.alg
obs = env.get_observations()
for rep in range(3):
    alg.storage.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    with torch.inference_mode():
        for _ in range(24):
            h0 = time.perf_counter()
            a = alg.act(obs, obs)
            obs, _, rew, dones, infos = env.step(a)
            alg.process_env_step(rew, dones, infos)
            host += time.perf_counter() - h0
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rep {rep}: host {host / 24 * 1e6:.1f} us/step (loop returned after {(t1 - t0) / 24 * 1e6:.1f} us/step), "
          f"wall incl. drain {(t2 - t0) / 24 * 1e6:.1f} us/step", flush=True)

# The update: host time to issue every launch of the 20 minibatches vs the update's wall time
# (which ends with the statistics readback, i.e. when the GPU has drained).  Issue time close to
# the wall time means the learn phase is launch-bound.
fused = getattr(alg, "_fused", None)
if fused is not None:
    for rep in range(3):
        alg.storage.clear()
        with torch.inference_mode():
            for _ in range(24):
                a = alg.act(obs, obs)
                obs, _, rew, dones, infos = env.step(a)
                alg.process_env_step(rew, dones, infos)
            alg.compute_returns(obs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        alg.update()
        t1 = time.perf_counter()
        print(f"update rep {rep}: host issue {fused.host_issue_s * 1e3:.2f} ms, wall {(t1 - t0) * 1e3:.2f} ms", flush=True)
