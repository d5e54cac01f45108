"""Policy evaluation (legged_gym/scripts/play.py:42-121, headless): load the latest checkpoint of
the task's experiment, optionally export the actor as TorchScript, run the policy, log robot 0's
states for the first 100 steps (utils/logger.py: the reference's 3 x 3 state figure, written as a
PNG next to the exported policy - headless, no viewer / camera) and print the average reward per
term over the first episode length, as play.py:73-121.

    python -m legged_gym_amd.scripts.play --task go1_rough [--load_run RUN --checkpoint IT] [--steps 1000]
"""
import os
import sys

import torch

import legged_gym_amd.envs  # noqa: F401
from legged_gym_amd import LEGGED_GYM_ROOT_DIR
from legged_gym_amd.utils import export_policy_as_jit, get_args, task_registry

EXPORT_POLICY = True


def play(args, steps=1000):
    env_cfg, train_cfg = task_registry.get_cfgs(name=args.task)
    env_cfg.env.num_envs = min(env_cfg.env.num_envs, 25)          # play.py:50-60 overrides
    env_cfg.terrain.num_rows = 5
    env_cfg.terrain.num_cols = 5
    env_cfg.terrain.curriculum = False
    env_cfg.noise.add_noise = False
    env_cfg.domain_rand.randomize_friction = False
    env_cfg.domain_rand.push_robots = False
    env_cfg.domain_rand.randomize_base_mass = False
    env_cfg.domain_rand.randomize_limb_mass = False
    env_cfg.commands.ranges.lin_vel_x = [0.5, 0.5]
    env_cfg.commands.ranges.lin_vel_y = [0.5, 0.5]
    env_cfg.commands.ranges.heading = [-1.57, -1.57]
    env, _ = task_registry.make_env(name=args.task, args=args, env_cfg=env_cfg)
    obs = env.get_observations()
    train_cfg.runner.resume = True
    ppo_runner, train_cfg = task_registry.make_alg_runner(env=env, name=args.task, args=args, train_cfg=train_cfg)
    policy = ppo_runner.get_inference_policy(device=env.device)
    if EXPORT_POLICY:
        path = os.path.join(LEGGED_GYM_ROOT_DIR, "logs", train_cfg.runner.experiment_name, "exported", "policies")
        export_policy_as_jit(ppo_runner.alg.actor_critic, path)
        print("Exported policy as jit script to: ", path)
    from legged_gym_amd.utils.logger import Logger
    logger = Logger(env.dt)
    robot_index, joint_index = 0, 1                       # play.py:73-77
    stop_state_log = min(100, steps - 1)
    stop_rew_log = min(int(env.max_episode_length) + 1, steps - 1)
    ep_rew = torch.zeros(env.num_envs, device=env.device)
    finished = []
    for i in range(steps):
        with torch.inference_mode():
            actions = policy(obs.detach())
            obs, _, rews, dones, infos = env.step(actions.detach())
        ep_rew += rews
        if dones.any():
            finished += ep_rew[dones].tolist()
            ep_rew[dones] = 0
        if i < stop_state_log:                            # play.py:94-109
            logger.log_states({
                "dof_pos_target": actions[robot_index, joint_index].item() * env.cfg.control.action_scale,
                "dof_pos": env.dof_pos[robot_index, joint_index].item(),
                "dof_vel": env.dof_vel[robot_index, joint_index].item(),
                "dof_torque": env.torques[robot_index, joint_index].item(),
                "command_x": env.commands[robot_index, 0].item(),
                "command_y": env.commands[robot_index, 1].item(),
                "command_yaw": env.commands[robot_index, 2].item(),
                "base_vel_x": env.base_lin_vel[robot_index, 0].item(),
                "base_vel_y": env.base_lin_vel[robot_index, 1].item(),
                "base_vel_z": env.base_lin_vel[robot_index, 2].item(),
                "base_vel_yaw": env.base_ang_vel[robot_index, 2].item(),
                "contact_forces_z": env.contact_forces[robot_index, env.feet_indices, 2].cpu().numpy(),
            })
        elif i == stop_state_log:
            png = logger.plot_states(os.path.join(path if EXPORT_POLICY else ".", "states.png"))
            print("State plots written to:", png)
        if 0 < i < stop_rew_log:                          # play.py:112-118
            if infos["episode"]:
                num_episodes = int(torch.sum(env.reset_buf).item())
                if num_episodes > 0:
                    logger.log_rewards(infos["episode"], num_episodes)
        elif i == stop_rew_log:
            logger.print_rewards()
    if finished:
        print(f"episodes: {len(finished)}  mean episode reward: {sum(finished) / len(finished):.3f}")
    return finished


if __name__ == "__main__":
    a = get_args()
    play(a, steps=int(os.environ.get("LGX_PLAY_STEPS", "1000")))
    sys.exit(0)
