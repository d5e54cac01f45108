"""Robot model assembly: robot JSON (tools/urdf_model.py) + env cfg -> `LgxModel`.

Replaces the Isaac Gym asset path of `_create_envs` (legged_robot.py:654-699): asset load,
DOF/body name queries, the POS drive setup with per-joint Kp/Kd from `cfg.control.stiffness`
(substring match on the DOF name, :693-699), and the asset/sim physics options.
"""
import json
import os

import numpy as np

from . import abi


class RobotAsset:
    def __init__(self, path):
        with open(path) as f:
            self.data = json.load(f)
        self.body_names = self.data["body_names"]
        self.dof_names = self.data["dof_names"]
        self.num_bodies = len(self.body_names)
        self.num_dof = len(self.dof_names)
        j = self.data["joints"]
        lower = np.array([x["lower"] for x in j], dtype=np.float64)
        upper = np.array([x["upper"] for x in j], dtype=np.float64)
        # URDF revolute joints without limits (lower == upper == 0, e.g. ANYmal-C) are free
        free = lower >= upper
        self.dof_lower = np.where(free, -1e3, lower)
        self.dof_upper = np.where(free, 1e3, upper)
        self.dof_has_limits = ~free
        self.dof_velocity = np.array([x["velocity"] for x in j], dtype=np.float64)
        self.dof_effort = np.array([x["effort"] for x in j], dtype=np.float64)
        self.nominal_mass = np.array([b["mass"] for b in self.data["dyn_bodies"]], dtype=np.float64)
        # dyn body of each reporting body (for randomised masses: reporting body i -> dyn body)
        self.report_dyn = [b["dyn_body"] for b in self.data["report_bodies"]]

    def find_bodies(self, pattern):
        return [i for i, n in enumerate(self.body_names) if pattern in n]


def build_model(asset: RobotAsset, cfg, sim_params):
    m = abi.LgxModel()
    d = asset.data
    for j, jt in enumerate(d["joints"]):
        for i in range(9):
            m.joint_rot[j][i] = jt["rot"][i]
        for i in range(3):
            m.joint_pos[j][i] = jt["pos"][i]
            m.joint_axis[j][i] = jt["axis"][i]
        m.dof_lower[j] = asset.dof_lower[j] if asset.dof_has_limits[j] else 0.0
        m.dof_upper[j] = asset.dof_upper[j] if asset.dof_has_limits[j] else 0.0
        m.dof_vel_limit[j] = jt["velocity"]
        m.dof_effort[j] = jt["effort"]
        kp = kd = 0.0
        for key, val in cfg.control.stiffness.items():  # legged_robot.py:693-699
            if key in asset.dof_names[j]:
                kp = float(val)
                kd = float(cfg.control.damping[key])
        m.kp[j] = kp
        m.kd[j] = kd
    for b, body in enumerate(d["dyn_bodies"]):
        m.body_mass[b] = body["mass"]
        for i in range(3):
            m.body_com[b][i] = body["com"][i]
        for i in range(6):
            m.body_inertia[b][i] = body["inertia"][i]
    pts = d["contact_points"]
    if len(pts) > abi.MAX_POINTS:
        raise ValueError(f"robot has {len(pts)} contact primitives > {abi.MAX_POINTS}")
    m.num_points = len(pts)
    m.num_report_bodies = asset.num_bodies
    m.leg_dof = int(d.get("leg_dof", 3))
    for i, p in enumerate(pts):
        for k in range(3):
            m.point_pos[i][k] = p["pos"][k]
        m.point_radius[i] = p["radius"]
        m.point_dyn[i] = p["dyn_body"]
        m.point_report[i] = p["report_body"]
    lg = cfg.sim.lgx
    m.contact_k, m.contact_c, m.friction_c = lg.contact_stiffness, lg.contact_damping, lg.friction_damping
    m.limit_k, m.limit_c = lg.limit_stiffness, lg.limit_damping
    m.ground_friction = cfg.terrain.static_friction
    g = sim_params.gravity
    for i in range(3):
        m.gravity[i] = 0.0 if cfg.asset.disable_gravity else g[i]
    m.sim_dt = np.float32(sim_params.dt)
    return m


def resolve_asset_path(path_template, root):
    return path_template.format(LEGGED_GYM_ROOT_DIR=root)


def load_actuator_net(path):
    """Actuator-net weights re-committed as data (.npz, exported by tools/export_actuator_nets.py)."""
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return dict(np.load(path, allow_pickle=False))
