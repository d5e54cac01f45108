"""LeggedRobot: the drop-in vectorised locomotion env, backed by the lgx HIP kernels.

Public surface = legged_gym/envs/base/legged_robot.py:51-975: constructor
`(cfg, sim_params, physics_engine, sim_device, headless)`, `step`, `reset`, `reset_idx`,
`post_physics_step`, `compute_observations`, the buffers rsl_rl and the play tools read
(obs_buf, rew_buf, reset_buf, episode_length_buf, extras, dof_pos, dof_vel, torques,
commands, base_lin_vel, base_ang_vel, contact_forces, feet_indices, dt, ...).

What runs where:
  * host (this file, setup only): config parsing, terrain, asset, domain randomisation
    tables, reward-term ordering, buffer allocation (torch), the C-ABI structs;
  * device (liblgx.so, one call per env step): `lgx_step` = clip + `decimation` fused physics
    substeps + actuator net + the fused post-physics kernel (termination, rewards, resets,
    observations) — no host synchronisation, no per-term launches.
"""
import ctypes as C
import os

import numpy as np
import torch

from legged_gym_amd import LEGGED_GYM_ROOT_DIR
from legged_gym_amd.envs.base.base_task import BaseTask
from legged_gym_amd.sim import abi
from legged_gym_amd.sim.model import RobotAsset, build_model, resolve_asset_path
from legged_gym_amd.utils.helpers import class_to_dict
from legged_gym_amd.utils.math import quat_rotate_inverse, torch_rand_float
from legged_gym_amd.utils.terrain import Terrain


def _ptr(t, ctype=abi.PF):
    return C.cast(C.c_void_p(t.data_ptr()), ctype) if t is not None else None


class LgxBackend:
    """Thin owner of one `lgx_sim` (product path: HIP only, no fallback)."""
    takes_actions = True   # step(counter, actions) reads the policy's tensor directly (lgx_step_from)

    def __init__(self, env, model, params, bufs):
        from legged_gym_amd.sim import lib as lgxlib
        if not str(env.device).startswith("cuda"):
            raise lgxlib.LgxError("the lgx engine runs on a GPU (sim_device=cuda:N with the GPU pipeline); "
                                  f"got device {env.device!r}")
        self.lib = lgxlib.load()
        self._check = lgxlib.check
        self.device = torch.device(env.device)
        self.handle = C.c_void_p()
        self._check(self.lib.lgx_sim_create(C.byref(model), C.byref(params), C.byref(bufs), self.device.index or 0,
                                            C.byref(self.handle)), "lgx_sim_create")

    def stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def step(self, counter, actions=None):
        if actions is None:
            self._check(self.lib.lgx_step(self.handle, counter, self.stream()), "lgx_step")
        else:
            self._check(self.lib.lgx_step_from(self.handle, C.c_void_p(actions.data_ptr()), counter, self.stream()),
                        "lgx_step_from")

    def simulate(self, n):
        self._check(self.lib.lgx_simulate(self.handle, n, self.stream()), "lgx_simulate")

    def drive_inputs(self, actions=None):
        self._check(self.lib.lgx_drive_inputs(self.handle, C.c_void_p(actions.data_ptr()) if actions is not None
                                              else None, self.stream()), "lgx_drive_inputs")

    def post_physics(self, counter, fused=False):
        if fused:   # the post-physics launch of lgx_step_from (with the Go1 actuator net when configured)
            self._check(self.lib.lgx_post_physics_fused(self.handle, counter, self.stream()), "lgx_post_physics_fused")
        else:
            self._check(self.lib.lgx_post_physics(self.handle, counter, self.stream()), "lgx_post_physics")

    def reset_idx(self, ids_i32, counter, init_done):
        self._check(self.lib.lgx_reset_idx(self.handle, C.c_void_p(ids_i32.data_ptr()), ids_i32.numel(), counter,
                                           int(init_done), self.stream()), "lgx_reset_idx")

    def rebind_obs(self, obs):
        self._check(self.lib.lgx_rebind_obs(self.handle, C.c_void_p(obs.data_ptr())), "lgx_rebind_obs")

    def sync_aux(self):
        self._check(self.lib.lgx_sync_aux(self.handle, self.stream()), "lgx_sync_aux")

    BUFFER_IDS = ("root_states", "dof_state", "dof_targets", "torques", "contact_forces", "actions",
                  "last_actions", "last_dof_vel", "last_root_vel", "commands", "base_lin_vel", "base_ang_vel",
                  "projected_gravity", "feet_air_time", "obs", "rew", "reset", "time_out", "episode_length",
                  "episode_sums", "measured_heights", "env_origins", "terrain_levels", "terrain_types", "extras")
    DTYPES = (torch.float32, torch.uint8, torch.int64)

    def buffer(self, name):
        """lgx_sim_buffer: (device pointer, shape, torch dtype) of a state tensor the sim writes
        (enum lgx_buffer_id order = BUFFER_IDS)."""
        ptr, shape, nd, dt = C.c_void_p(), (C.c_int64 * 4)(), C.c_int32(), C.c_int32()
        self._check(self.lib.lgx_sim_buffer(self.handle, self.BUFFER_IDS.index(name), C.byref(ptr), shape,
                                            C.byref(nd), C.byref(dt)), "lgx_sim_buffer")
        return ptr.value or 0, tuple(shape[:nd.value]), self.DTYPES[dt.value]

    def rebind_extras(self, snapshot):
        self._check(self.lib.lgx_rebind_extras(self.handle, C.c_void_p(snapshot.data_ptr())), "lgx_rebind_extras")

    def set_draws(self, draws):
        self._check(self.lib.lgx_set_draws(self.handle, C.c_void_p(draws.data_ptr()) if draws is not None else None),
                    "lgx_set_draws")

    def close(self):
        if self.handle:
            self.lib.lgx_sim_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LeggedRobot(BaseTask):
    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.cfg = cfg
        self.sim_params = sim_params
        self.height_samples = None
        self.debug_viz = False
        self.init_done = False
        self._parse_cfg(self.cfg)
        super().__init__(self.cfg, sim_params, physics_engine, sim_device, headless)
        self._init_buffers()
        self._prepare_reward_function()
        self._build_lgx()
        self.init_done = True

    # ------------------------------------------------------------------ step path
    def step(self, actions):
        """legged_robot.py:79-107 as one C-ABI call (lgx_step)."""
        self._next_obs_buffer()
        snap = self._next_extras_snapshot()
        self.common_step_counter += 1
        if self._direct_actions(actions):      # kernel reads the policy's tensor, clips into self.actions
            self._backend.step(self.common_step_counter, actions)
        else:
            self.actions.copy_(actions)        # clipped in place by the kernel (:85-86)
            self._backend.step(self.common_step_counter)
        self._publish_extras(snap)
        return self.obs_buf, self.privileged_obs_buf, self.rew_buf, self.reset_buf, self.extras

    def post_physics_step(self, fused=False):
        """legged_robot.py:109-141 on the current physics state (no physics).  fused=True issues it
        as `step` does after its physics launch (lgx_post_physics_fused: the Go1 actuator net over
        this step's model_ins in the same launch)."""
        self._next_obs_buffer()
        snap = self._next_extras_snapshot()
        self.common_step_counter += 1
        if fused:
            self._backend.post_physics(self.common_step_counter, fused=True)
        else:
            self._backend.post_physics(self.common_step_counter)
        self._publish_extras(snap)

    def simulate(self, n=1):
        """n physics substeps with the current `target_poses` (gym.simulate x n)."""
        self._backend.simulate(n)

    def reset_idx(self, env_ids):
        """legged_robot.py:150-193 for an explicit list of envs."""
        if len(env_ids) == 0:
            return
        ids = torch.as_tensor(env_ids, device=self.device).to(torch.int32).contiguous()
        snap = self._next_extras_snapshot()
        self._backend.reset_idx(ids, self.common_step_counter, self.init_done)
        self._publish_extras(snap)

    def _next_obs_buffer(self):
        """Alternate between two observation buffers: the reference returns a fresh obs tensor per
        step (legged_robot.py:218), and rsl_rl keeps the previous one until process_env_step."""
        self._obs_slot ^= 1
        ob = self._obs_bufs[self._obs_slot]
        self._lgx_bufs.obs = _ptr(ob)
        if hasattr(self._backend, "rebind_obs"):
            self._backend.rebind_obs(ob)
        self.obs_buf = ob

    def compute_observations(self):
        raise NotImplementedError("observations are produced inside lgx_step/lgx_post_physics")

    def _direct_actions(self, actions):
        return (getattr(self._backend, "takes_actions", False) and isinstance(actions, torch.Tensor)
                and actions.device == self.actions.device and actions.dtype == torch.float32
                and actions.shape == self.actions.shape and actions.is_contiguous())

    def _next_extras_snapshot(self):
        """A fresh [T + 2] tensor the kernels fill with this call's extras (lgx_rebind_extras);
        None when the backend has no such output (then _publish_extras clones)."""
        if not hasattr(self._backend, "rebind_extras"):
            return None
        snap = torch.empty_like(self._extras_buf)
        self._backend.rebind_extras(snap)
        return snap

    def _publish_extras(self, snap=None):
        """extras["episode"] / ["time_outs"] (legged_robot.py:182-193).  The device keeps the
        reference's stale-until-next-reset semantics; every call publishes its own snapshot
        (written by the finalize kernel, or cloned) so that consumers that keep references
        (rsl_rl ep_infos) see per-step values."""
        if snap is None:
            snap = self._extras_buf.clone()
        ep = {}
        for key, row in self._extras_rows:
            ep[key] = snap[row]
        self.extras["episode"] = ep
        if self.cfg.env.send_timeouts:
            self.extras["time_outs"] = self._extras_time_outs

    # ------------------------------------------------------------------ setup
    def _parse_cfg(self, cfg):  # legged_robot.py:769-779
        self.dt = self.cfg.control.decimation * self.sim_params.dt
        self.obs_scales = self.cfg.normalization.obs_scales
        self.reward_scales = class_to_dict(self.cfg.rewards.scales)
        self.command_ranges = class_to_dict(self.cfg.commands.ranges)
        if self.cfg.terrain.mesh_type not in ["heightfield", "trimesh"]:
            self.cfg.terrain.curriculum = False
        self.max_episode_length_s = self.cfg.env.episode_length_s
        self.max_episode_length = np.ceil(self.max_episode_length_s / self.dt)
        self.cfg.domain_rand.push_interval = np.ceil(self.cfg.domain_rand.push_interval_s / self.dt)

    def create_sim(self):  # legged_robot.py:233-249
        self.up_axis_idx = 2
        mesh_type = self.cfg.terrain.mesh_type
        if mesh_type in ["heightfield", "trimesh"]:
            self.terrain = Terrain(self.cfg.terrain, self.num_envs)
            hs = self.terrain.heightsamples
            self.height_samples = torch.tensor(hs).view(self.terrain.tot_rows, self.terrain.tot_cols).to(self.device)
        elif mesh_type not in [None, "none", "plane"]:
            raise ValueError("Terrain mesh type not recognised. Allowed types are [None, plane, heightfield, trimesh]")
        self._create_envs()

    def _create_envs(self):  # legged_robot.py:645-740
        path = resolve_asset_path(self.cfg.asset.file, LEGGED_GYM_ROOT_DIR)
        self.asset = RobotAsset(path)
        self.num_dof = self.asset.num_dof
        self.num_bodies = self.asset.num_bodies
        self.dof_names = self.asset.dof_names
        self.num_dofs = len(self.dof_names)
        body_names = self.asset.body_names
        feet_names = [s for s in body_names if self.cfg.asset.foot_name in s]
        penalized = [s for name in self.cfg.asset.penalize_contacts_on for s in body_names if name in s]
        terminate = [s for name in self.cfg.asset.terminate_after_contacts_on for s in body_names if name in s]
        init = self.cfg.init_state
        self.base_init_state = torch.tensor(init.pos + init.rot + init.lin_vel + init.ang_vel, dtype=torch.float,
                                            device=self.device)
        self._get_env_origins()
        self._process_dof_props()
        # the reference's per-env creation loop (legged_robot.py:707-728) draws each env's start
        # pose offset (torch, on self.device; the pose itself is overwritten by the first reset)
        # and builds the friction tables (CPU torch generator) right after env 0's draw: keep
        # that consumption order so the same seed gives the same friction buckets
        if str(self.device) == "cpu":
            torch_rand_float(-1., 1., (2, 1), device=self.device)
            self._process_rigid_shape_props()
            for _ in range(1, self.num_envs):
                torch_rand_float(-1., 1., (2, 1), device=self.device)
        else:
            self._process_rigid_shape_props()
        self._process_rigid_body_props()
        idx = lambda names: torch.tensor([body_names.index(n) for n in names], dtype=torch.long, device=self.device)
        self.feet_indices = idx(feet_names)
        self.penalised_contact_indices = idx(penalized)
        self.termination_contact_indices = idx(terminate)

    def _process_rigid_shape_props(self):  # legged_robot.py:259-282: 64 friction buckets
        if self.cfg.domain_rand.randomize_friction:
            lo, hi = self.cfg.domain_rand.friction_range
            bucket_ids = torch.randint(0, 64, (self.num_envs, 1))
            buckets = torch_rand_float(lo, hi, (64, 1), device="cpu")
            self.friction_coeffs = buckets[bucket_ids].view(self.num_envs)
        else:
            self.friction_coeffs = torch.ones(self.num_envs)
        self.friction_coeffs = self.friction_coeffs.to(self.device, torch.float)

    def _process_dof_props(self):  # legged_robot.py:284-310
        lo = torch.tensor(self.asset.dof_lower, dtype=torch.float, device=self.device)
        hi = torch.tensor(self.asset.dof_upper, dtype=torch.float, device=self.device)
        m, r = (lo + hi) / 2, hi - lo
        s = self.cfg.rewards.soft_dof_pos_limit
        self.dof_pos_limits = torch.stack([m - 0.5 * r * s, m + 0.5 * r * s], dim=1)
        self.dof_vel_limits = torch.tensor(self.asset.dof_velocity, dtype=torch.float, device=self.device)
        self.torque_limits = torch.tensor(self.asset.dof_effort, dtype=torch.float, device=self.device)

    def _process_rigid_body_props(self):  # legged_robot.py:312-335 (+ recomputeInertia, :726)
        """Per-env mass scale of each dynamic body.  Reporting-body masses are randomised as in
        the reference (base: +U(range) kg, other bodies: x(1+U(pct))); inertia scales with mass."""
        rb = self.asset.data["report_bodies"]
        masses = np.array([b["mass"] for b in rb], dtype=np.float64)
        rnd = np.tile(masses, (self.num_envs, 1))
        dr = self.cfg.domain_rand
        # numpy draws in the reference's order: env-major, body 0 (base) then bodies 1.. (limbs);
        # np.random.uniform(lo, hi) == lo + (hi - lo) * random_sample()
        cols = ([0] if dr.randomize_base_mass else []) + (list(range(1, len(rb))) if dr.randomize_limb_mass else [])
        if cols:
            u = np.random.random_sample((self.num_envs, len(cols)))
            for j, bi in enumerate(cols):
                if bi == 0:
                    lo, hi = dr.added_mass_range
                    rnd[:, 0] += lo + (hi - lo) * u[:, j]
                else:
                    lo, hi = dr.added_limb_percentage
                    rnd[:, bi] *= 1 + (lo + (hi - lo) * u[:, j])
        self.body_masses = rnd   # [N, reporting bodies] after randomisation (float64, as set on the actor)
        dyn_mass = np.zeros((self.num_envs, abi.NUM_DYN))
        for i, b in enumerate(rb):
            dyn_mass[:, b["dyn_body"]] += rnd[:, i]
        scale = dyn_mass / np.maximum(self.asset.nominal_mass, 1e-12)
        self.body_mass_scale = torch.tensor(scale, dtype=torch.float, device=self.device)

    def _get_env_origins(self):  # legged_robot.py:742-767
        N, dev = self.num_envs, self.device
        if self.cfg.terrain.mesh_type in ["heightfield", "trimesh"]:
            self.custom_origins = True
            self.env_origins = torch.zeros(N, 3, device=dev)
            max_init_level = self.cfg.terrain.max_init_terrain_level
            if not self.cfg.terrain.curriculum:
                max_init_level = self.cfg.terrain.num_rows - 1
            self.terrain_levels = torch.randint(0, max_init_level + 1, (N,), device=dev)
            self.terrain_types = torch.div(torch.arange(N, device=dev), (N / self.cfg.terrain.num_cols),
                                           rounding_mode="floor").to(torch.long)
            self.max_terrain_level = self.cfg.terrain.num_rows
            self.terrain_origins = torch.from_numpy(self.terrain.env_origins).to(dev).to(torch.float).contiguous()
            self.env_origins[:] = self.terrain_origins[self.terrain_levels, self.terrain_types]
        else:
            self.custom_origins = False
            self.env_origins = torch.zeros(N, 3, device=dev)
            num_cols = np.floor(np.sqrt(N))
            num_rows = np.ceil(N / num_cols)
            xx, yy = torch.meshgrid(torch.arange(num_rows), torch.arange(num_cols), indexing="ij")
            spacing = self.cfg.env.env_spacing
            self.env_origins[:, 0] = spacing * xx.flatten()[:N].to(dev)
            self.env_origins[:, 1] = spacing * yy.flatten()[:N].to(dev)
            self.terrain_levels = torch.zeros(N, dtype=torch.long, device=dev)
            self.terrain_types = torch.zeros(N, dtype=torch.long, device=dev)
            self.terrain_origins = torch.zeros(1, 1, 3, device=dev)
            self.max_terrain_level = 1

    def _init_buffers(self):  # legged_robot.py:503-572
        N, dev, na = self.num_envs, self.device, self.num_actions
        f = dict(dtype=torch.float, device=dev)
        self.root_states = torch.zeros(N, 13, **f)
        self.root_states[:] = self.base_init_state
        self.root_states[:, :3] += self.env_origins
        self.dof_state = torch.zeros(N * self.num_dof, 2, **f)
        self.dof_pos = self.dof_state.view(N, self.num_dof, 2)[..., 0]
        self.dof_vel = self.dof_state.view(N, self.num_dof, 2)[..., 1]
        self.base_quat = self.root_states[:, 3:7]
        self.contact_forces = torch.zeros(N, abi.MAX_BODIES, 3, **f)[:, :self.num_bodies]
        self._contact_forces_full = self.contact_forces
        self.common_step_counter = 0
        self.extras = {}
        self.noise_scale_vec = self._get_noise_scale_vec(self.cfg)
        self.gravity_vec = torch.tensor([0.0, 0.0, -1.0], **f).repeat((N, 1))
        self.forward_vec = torch.tensor([1.0, 0.0, 0.0], **f).repeat((N, 1))
        self.target_poses = torch.zeros(N, na, **f)
        self.torques = torch.zeros(N, na, **f)
        self.p_gains = torch.zeros(na, **f)
        self.d_gains = torch.zeros(na, **f)
        self.actions = torch.zeros(N, na, **f)
        self.last_actions = torch.zeros(N, na, **f)
        self.last_dof_vel = torch.zeros(N, self.num_dof, **f)
        self.last_root_vel = torch.zeros(N, 6, **f)
        self.commands = torch.zeros(N, self.cfg.commands.num_commands, **f)
        self.commands_scale = torch.tensor([self.obs_scales.lin_vel, self.obs_scales.lin_vel, self.obs_scales.ang_vel], **f)
        # the kernels keep 4 slots per env (lgx.h feet_air_time [N,4]); the biped uses the first 2
        self._feet_air_time_full = torch.zeros(N, 4, **f)
        self.feet_air_time = self._feet_air_time_full[:, :self.feet_indices.shape[0]]
        self.last_contacts = torch.zeros(N, len(self.feet_indices), dtype=torch.bool, device=dev)
        self.base_lin_vel = quat_rotate_inverse(self.base_quat, self.root_states[:, 7:10]).contiguous()
        self.base_ang_vel = quat_rotate_inverse(self.base_quat, self.root_states[:, 10:13]).contiguous()
        self.projected_gravity = quat_rotate_inverse(self.base_quat, self.gravity_vec).contiguous()
        if self.cfg.terrain.measure_heights:
            self.height_points = self._init_height_points()
        else:
            self.num_height_points = 0
        self.measured_heights = torch.zeros(N, max(self.num_height_points, 1), **f)
        self.default_dof_pos = torch.zeros(self.num_dof, **f)
        for i, name in enumerate(self.dof_names):
            self.default_dof_pos[i] = self.cfg.init_state.default_joint_angles[name]
            found = False
            for key in self.cfg.control.stiffness.keys():
                if key in name:
                    self.p_gains[i] = self.cfg.control.stiffness[key]
                    self.d_gains[i] = self.cfg.control.damping[key]
                    found = True
            if not found and self.cfg.control.control_type in ["P", "V"]:
                print(f"PD gain of joint {name} were not defined, setting them to zero")
        self.default_dof_pos = self.default_dof_pos.unsqueeze(0)

    def _get_noise_scale_vec(self, cfg):  # legged_robot.py:477-500
        nv = torch.zeros_like(self.obs_buf[0])
        self.add_noise = self.cfg.noise.add_noise
        ns, nl, os_ = self.cfg.noise.noise_scales, self.cfg.noise.noise_level, self.obs_scales
        nv[:3] = ns.lin_vel * nl * os_.lin_vel
        nv[3:6] = ns.ang_vel * nl * os_.ang_vel
        nv[6:9] = ns.gravity * nl
        nv[9:12] = 0.0
        nv[12:24] = ns.dof_pos * nl * os_.dof_pos
        nv[24:36] = ns.dof_vel * nl * os_.dof_vel
        nv[36:48] = 0.0
        if self.cfg.terrain.measure_heights:
            nv[48:235] = ns.height_measurements * nl * os_.height_measurements
        return nv

    def _init_height_points(self):  # legged_robot.py:802-816
        y = torch.tensor(self.cfg.terrain.measured_points_y, device=self.device)
        x = torch.tensor(self.cfg.terrain.measured_points_x, device=self.device)
        gx, gy = torch.meshgrid(x, y, indexing="ij")
        self.num_height_points = gx.numel()
        pts = torch.zeros(self.num_envs, self.num_height_points, 3, device=self.device)
        pts[:, :, 0] = gx.flatten()
        pts[:, :, 1] = gy.flatten()
        return pts

    def _prepare_reward_function(self):  # legged_robot.py:574-598
        for key in list(self.reward_scales.keys()):
            if self.reward_scales[key] == 0:
                self.reward_scales.pop(key)
            else:
                self.reward_scales[key] *= self.dt
        self.reward_names = []
        for name in self.reward_scales.keys():
            if name == "termination":
                continue
            if name not in abi.REWARD_IDS:
                raise AttributeError(f"'{type(self).__name__}' has no reward term '_reward_{name}'")
            self.reward_names.append(name)
        rows = self.reward_names + (["termination"] if "termination" in self.reward_scales else [])
        self._episode_sums_buf = torch.zeros(max(len(rows), 1), self.num_envs, dtype=torch.float, device=self.device)
        # dict keys in the reference's order (reward_scales: alphabetical, "termination" in its place,
        # legged_robot.py:596-597); buffer rows: the terms in evaluation order, then termination
        self.episode_sums = {name: self._episode_sums_buf[rows.index(name)] for name in self.reward_scales}
        # extras rows: one per episode-sum row (alphabetical key order as the reference dict)
        T = len(rows)
        self._extras_buf = torch.zeros(T + 2, dtype=torch.float, device=self.device)
        order = [k for k in self.reward_scales.keys()]
        self._extras_rows = [("rew_" + k, rows.index(k)) for k in order]
        if self.cfg.terrain.curriculum:
            self._extras_rows.append(("terrain_level", T))
        self._extras_time_outs = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)

    # ------------------------------------------------------------------ C-ABI structs
    def _actuator_setup(self, params, bufs):
        """Robot-specific actuator-net state (Go1 overrides)."""
        return None

    def _control_type(self):
        # the reference step path drives joints through PhysX position drives (legged_robot.py:93-96);
        # cfg.control.explicit_torques selects its commented-out explicit path, _compute_torques
        # (legged_robot.py:90-91,370-392), with control_type P | V | T
        if getattr(self.cfg.control, "explicit_torques", False):
            return abi.CTRL[self.cfg.control.control_type]
        return abi.CTRL["POS_DRIVE"]

    def _build_lgx(self):
        cfg, N = self.cfg, self.num_envs
        self._lgx_model = build_model(self.asset, cfg, self.sim_params)
        p = abi.LgxEnvParams()
        p.num_envs, p.num_obs, p.decimation = N, self.num_obs, cfg.control.decimation
        p.control_type = self._control_type()
        p.action_scale = cfg.control.action_scale
        p.clip_actions = cfg.normalization.clip_actions
        p.clip_obs = cfg.normalization.clip_observations
        p.dt = self.dt
        dd = self.default_dof_pos[0].cpu().numpy()
        lims = self.dof_pos_limits.cpu().numpy()
        for j in range(abi.NUM_DOF):
            p.default_dof_pos[j] = dd[j]
            p.soft_lower[j], p.soft_upper[j] = lims[j, 0], lims[j, 1]
            p.dof_vel_limits[j] = float(self.dof_vel_limits[j])
            p.torque_limits[j] = float(self.torque_limits[j])
            p.p_gains[j], p.d_gains[j] = float(self.p_gains[j]), float(self.d_gains[j])
        p.soft_dof_vel_limit = cfg.rewards.soft_dof_vel_limit
        p.soft_torque_limit = cfg.rewards.soft_torque_limit
        p.max_episode_length = self.max_episode_length
        p.max_episode_length_s = self.max_episode_length_s
        p.resample_interval = int(cfg.commands.resampling_time / self.dt)
        p.push_robots = int(bool(cfg.domain_rand.push_robots))
        p.push_interval = int(cfg.domain_rand.push_interval)
        p.max_push_vel_xy = cfg.domain_rand.max_push_vel_xy
        p.heading_command = int(bool(cfg.commands.heading_command))
        for k, name in enumerate(["lin_vel_x", "lin_vel_y", "ang_vel_yaw", "heading"]):
            p.cmd_ranges[k][0], p.cmd_ranges[k][1] = self.command_ranges[name]
        os_ = self.obs_scales
        p.obs_scale_lin_vel, p.obs_scale_ang_vel = os_.lin_vel, os_.ang_vel
        p.obs_scale_dof_pos, p.obs_scale_dof_vel, p.obs_scale_height = os_.dof_pos, os_.dof_vel, os_.height_measurements
        p.add_noise = int(bool(self.add_noise))
        nv = self.noise_scale_vec.cpu().numpy()
        for i in range(self.num_obs):
            p.noise_scale_vec[i] = nv[i]
        p.terrain_kind = 1 if self.height_samples is not None else 0
        p.measure_heights = int(bool(cfg.terrain.measure_heights))
        p.num_height_points = self.num_height_points
        if cfg.terrain.measure_heights:
            hp = self.height_points[0].cpu().numpy()
            for i in range(self.num_height_points):
                p.height_points[i][0], p.height_points[i][1] = hp[i, 0], hp[i, 1]
        p.border_size, p.horizontal_scale, p.vertical_scale = (cfg.terrain.border_size, cfg.terrain.horizontal_scale,
                                                               cfg.terrain.vertical_scale)
        p.curriculum = int(bool(cfg.terrain.curriculum))
        p.custom_origins = int(self.custom_origins)
        p.max_terrain_level = self.max_terrain_level
        p.terrain_num_cols = cfg.terrain.num_cols if self.custom_origins else 1
        p.terrain_env_length = self.terrain.env_length if self.custom_origins else 0.0
        for i in range(13):
            p.base_init_state[i] = float(self.base_init_state[i])
        p.num_terms = len(self.reward_names)
        for t, name in enumerate(self.reward_names):
            p.term_ids[t] = abi.REWARD_IDS[name]
            p.term_scales[t] = self.reward_scales[name]
        p.termination_slot = len(self.reward_names) if "termination" in self.reward_scales else -1
        p.termination_scale = self.reward_scales.get("termination", 0.0)
        p.only_positive_rewards = int(bool(cfg.rewards.only_positive_rewards))
        p.tracking_sigma = cfg.rewards.tracking_sigma
        p.base_height_target = cfg.rewards.base_height_target
        p.max_contact_force = cfg.rewards.max_contact_force
        for name, cnt, arr, src in (("feet", "num_feet", "feet_indices", self.feet_indices),
                                    ("pen", "num_penalised", "penalised_indices", self.penalised_contact_indices),
                                    ("term", "num_termination_bodies", "termination_indices",
                                     self.termination_contact_indices)):
            vals = src.cpu().tolist()
            if len(vals) > len(getattr(p, arr)):
                raise ValueError(f"too many {name} bodies")
            setattr(p, cnt, len(vals))
            for i, v in enumerate(vals):
                getattr(p, arr)[i] = v
        p.send_timeouts = int(bool(cfg.env.send_timeouts))
        p.seed = int(getattr(cfg, "seed", 1)) & 0xFFFFFFFFFFFFFFFF
        self._scratch = torch.zeros(int(self._scratch_floats()), dtype=torch.float, device=self.device)
        b = abi.LgxBuffers()
        for field, t in (("root_states", self.root_states), ("dof_state", self.dof_state),
                         ("dof_targets", self.target_poses), ("torques", self.torques),
                         ("contact_forces", self._contact_forces_full), ("actions", self.actions),
                         ("last_actions", self.last_actions), ("last_dof_vel", self.last_dof_vel),
                         ("last_root_vel", self.last_root_vel), ("commands", self.commands),
                         ("base_lin_vel", self.base_lin_vel), ("base_ang_vel", self.base_ang_vel),
                         ("projected_gravity", self.projected_gravity), ("feet_air_time", self._feet_air_time_full),
                         ("obs", self.obs_buf), ("rew", self.rew_buf), ("episode_sums", self._episode_sums_buf),
                         ("measured_heights", self.measured_heights), ("env_origins", self.env_origins),
                         ("terrain_origins", self.terrain_origins), ("body_mass_scale", self.body_mass_scale),
                         ("friction", self.friction_coeffs), ("extras", self._extras_buf), ("scratch", self._scratch)):
            assert t.is_contiguous() or field == "contact_forces", field
            setattr(b, field, _ptr(t))
        b.reset = _ptr(self.reset_buf, abi.PU8)
        b.time_out = _ptr(self.time_out_buf, abi.PU8)
        b.extras_time_outs = _ptr(self._extras_time_outs, abi.PU8)
        b.episode_length = _ptr(self._episode_length_buf, abi.PI64)
        b.terrain_levels = _ptr(self.terrain_levels, abi.PI64)
        b.terrain_types = _ptr(self.terrain_types, abi.PI64)
        if self.height_samples is not None:
            self.height_samples = self.height_samples.contiguous()
            b.height_samples = _ptr(self.height_samples, abi.PI16)
            b.hf_rows, b.hf_cols = self.height_samples.shape
            self.hf_trimesh = self._trimesh_contact_table()
            if self.hf_trimesh is not None:
                b.hf_trimesh = C.cast(C.c_void_p(self.hf_trimesh.data_ptr()), C.POINTER(C.c_int8))
        self._actuator_setup(p, b)
        self._lgx_params, self._lgx_bufs = p, b
        self._obs_bufs = [self.obs_buf, torch.zeros_like(self.obs_buf)]
        self._obs_slot = 0
        self._backend = self._make_backend(self._lgx_model, p, b)

    def _trimesh_contact_table(self):
        """mesh_type 'trimesh' with a slope threshold: the contact table of the slope-corrected mesh
        (terrain.py:70-73) - built on the device by lgx_trimesh_build on the GPU path, from the
        numpy restatement (utils/terrain.py) for CPU tensors (the oracle backend).  None: contact
        against the heightfield itself (mesh_type 'heightfield': PhysX heightfield, no correction)."""
        tcfg = self.cfg.terrain
        if tcfg.mesh_type != "trimesh" or getattr(tcfg, "slope_treshold", None) is None:
            return None
        mode = os.environ.get("LGX_TRIMESH", "1")       # A/B switches: 0 = contact on the raw heightfield,
        if mode == "0":                                  # 2 = table bound but no cell flagged
            return None
        R, Cc = self.height_samples.shape
        thr = tcfg.slope_treshold * (tcfg.horizontal_scale / tcfg.vertical_scale)   # (the library's scaling)
        if self.height_samples.is_cuda:
            from legged_gym_amd.sim import lib as lgxlib
            lib = lgxlib.load()
            table = torch.empty(R, Cc, dtype=torch.int8, device=self.device)
            lgxlib.check(lib.lgx_trimesh_build(C.c_void_p(self.height_samples.data_ptr()), R, Cc, tcfg.horizontal_scale,
                                               tcfg.vertical_scale, thr, None, None, C.c_void_p(table.data_ptr()),
                                               C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                         "lgx_trimesh_build")
            if mode == "2":
                table &= 15
            return table
        from legged_gym_amd.utils.terrain import trimesh_contact_tables, trimesh_vertex_moves
        dx, dy = trimesh_vertex_moves(self.height_samples.cpu().numpy(), tcfg.horizontal_scale, tcfg.vertical_scale,
                                      tcfg.slope_treshold)
        code, flag = trimesh_contact_tables(dx, dy)
        return torch.from_numpy((code | (flag << 4)).astype(np.int8)).to(self.device)

    def _scratch_floats(self):
        blocks = (self.num_envs + abi.ENV_BLOCK - 1) // abi.ENV_BLOCK  # >= lgx_scratch_floats()
        return blocks * (abi.MAX_TERMS + 2) + 64

    def _make_backend(self, model, params, bufs):
        return LgxBackend(self, model, params, bufs)
