"""BaseTask: buffer allocation, device choice, reset() and the VecEnv observation getters.

Mirrors legged_gym/envs/base/base_task.py:38-115.  The viewer (render, :120-144) has no
counterpart: the lgx engine is headless; `render()` is a no-op kept for API compatibility.
"""
import torch


def parse_device_str(device):
    kind, _, idx = device.partition(":")
    return kind, int(idx) if idx else 0


class BaseTask:
    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.sim_params = sim_params
        self.physics_engine = physics_engine
        self.sim_device = sim_device
        sim_device_type, self.sim_device_id = parse_device_str(sim_device)
        self.headless = headless
        # base_task.py:49-54: env tensors live on the sim device with the GPU pipeline
        if sim_device_type == "cuda" and sim_params.use_gpu_pipeline:
            self.device = sim_device
        else:
            self.device = "cpu"
        self.graphics_device_id = -1 if headless else self.sim_device_id

        self.num_envs = cfg.env.num_envs
        self.num_obs = cfg.env.num_observations
        self.num_privileged_obs = cfg.env.num_privileged_obs
        self.num_actions = cfg.env.num_actions

        N, dev = self.num_envs, self.device
        self.obs_buf = torch.zeros(N, self.num_obs, device=dev, dtype=torch.float)
        self.rew_buf = torch.zeros(N, device=dev, dtype=torch.float)
        # reference: long ones before the first step, bool afterwards (base_task.py:72 vs
        # legged_robot.py:146); here a bool buffer bound to the kernels from the start
        self.reset_buf = torch.ones(N, device=dev, dtype=torch.bool)
        self._episode_length_buf = torch.zeros(N, device=dev, dtype=torch.long)
        self.time_out_buf = torch.zeros(N, device=dev, dtype=torch.bool)
        if self.num_privileged_obs is not None:
            self.privileged_obs_buf = torch.zeros(N, self.num_privileged_obs, device=dev, dtype=torch.float)
        else:
            self.privileged_obs_buf = None
        self.extras = {}
        self.create_sim()
        self.enable_viewer_sync = True
        self.viewer = None

    # rsl_rl writes `env.episode_length_buf = randint_like(...)` (init_at_random_ep_len): keep
    # the kernel-bound storage and copy into it
    @property
    def episode_length_buf(self):
        return self._episode_length_buf

    @episode_length_buf.setter
    def episode_length_buf(self, value):
        self._episode_length_buf.copy_(value.to(self._episode_length_buf.device, torch.long))

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def reset_idx(self, env_ids):
        raise NotImplementedError

    def reset(self):
        """base_task.py:111-115: reset all envs, then one zero-action step."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, privileged_obs, _, _, _ = self.step(torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs, privileged_obs

    def step(self, actions):
        raise NotImplementedError

    def render(self, sync_frame_time=True):
        return None
