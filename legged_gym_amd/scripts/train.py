"""Training entry point (legged_gym/scripts/train.py:31-47): make_env -> make_alg_runner -> learn.

    python -m legged_gym_amd.scripts.train --task go1_rough --headless [--num_envs N] [--max_iterations K]
Multi-GPU (one rank per GPU, RCCL gradient all-reduce):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m legged_gym_amd.scripts.train ...
"""
import os

import torch

import legged_gym_amd.envs  # noqa: F401  (task registrations)
from legged_gym_amd.utils import get_args, task_registry


def train(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        args.sim_device = args.rl_device = f"cuda:{local}"
        args.seed = (args.seed if args.seed is not None else 1) + dist.get_rank()
    env, env_cfg = task_registry.make_env(name=args.task, args=args)
    log_root = None if (world > 1 and int(os.environ.get("RANK", "0")) != 0) else "default"
    ppo_runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args, log_root=log_root)
    try:
        ppo_runner.learn(num_learning_iterations=train_cfg.runner.max_iterations, init_at_random_ep_len=True)
    finally:
        ppo_runner.close()
        if world > 1:
            torch.distributed.destroy_process_group()


if __name__ == "__main__":
    train(get_args())
