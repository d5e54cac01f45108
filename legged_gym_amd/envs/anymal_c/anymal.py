"""ANYmal-C env (legged_gym/envs/anymal_c/anymal.py:46-80).

The SEA LSTM actuator network is only reachable through the reference's `_compute_torques`
(anymal.py:71-78), which this fork's step path does not call (the step uses the PhysX position
drive, legged_robot.py:93-96).  Here it is an opt-in torque source of the step itself:
`cfg.control.explicit_torques = True` with `use_actuator_network = True` (the C5 config's default)
runs the LSTM inside the physics launch once per substep (LGX_CTRL_SEA: input
[a * action_scale + q0 - q, qd] x in_scale, torque = out_scale * Linear(h), clamped to the URDF
effort limit as PhysX's effort-mode drive does), its hidden / cell state [2, N*12, 8] in
`sea_hidden_state` / `sea_cell_state` and zeroed for envs that reset (anymal.py:56-60).
`actuator_torques()` runs one LSTM step on its own (lgx_actuator_lstm, HIP).
"""
import ctypes as C

import numpy as np
import torch

from legged_gym_amd import LEGGED_GYM_ROOT_DIR
from legged_gym_amd.envs.base.legged_robot import LeggedRobot
from legged_gym_amd.sim.model import load_actuator_net


def pack_lstm_weights(net):
    order = ["in_scale", "out_scale", "w_ih_l0", "w_hh_l0", "b_ih_l0", "b_hh_l0", "w_ih_l1", "w_hh_l1", "b_ih_l1",
             "b_hh_l1", "w_lin", "b_lin"]
    return np.concatenate([np.asarray(net[k], np.float32).ravel() for k in order])


class Anymal(LeggedRobot):
    def _sea_control(self):
        return getattr(self.cfg.control, "explicit_torques", False) and \
            getattr(self.cfg.control, "use_actuator_network", False)

    def _control_type(self):
        # explicit torques = the reference's Anymal._compute_torques: the SEA LSTM when
        # use_actuator_network is set (anymal.py:71-78), else LeggedRobot's P / V / T law
        if self._sea_control():
            from legged_gym_amd.sim import abi
            return abi.CTRL["SEA"]
        return LeggedRobot._control_type(self)

    def _actuator_setup(self, params, bufs):
        if self._sea_control():
            from legged_gym_amd.envs.base.legged_robot import _ptr
            bufs.sea_w = _ptr(self.actuator_net_weights)
            bufs.sea_h = _ptr(self.sea_hidden_state)
            bufs.sea_c = _ptr(self.sea_cell_state)
        return super()._actuator_setup(params, bufs)

    def _init_buffers(self):
        super()._init_buffers()
        M = self.num_envs * self.num_actions
        self.sea_input = torch.zeros(M, 1, 2, device=self.device)
        self.sea_hidden_state = torch.zeros(2, M, 8, device=self.device)
        self.sea_cell_state = torch.zeros(2, M, 8, device=self.device)
        self.sea_hidden_state_per_env = self.sea_hidden_state.view(2, self.num_envs, self.num_actions, 8)
        self.sea_cell_state_per_env = self.sea_cell_state.view(2, self.num_envs, self.num_actions, 8)
        self._sea_tau = torch.zeros(M, device=self.device)
        if getattr(self.cfg.control, "use_actuator_network", False):
            net = load_actuator_net(self.cfg.control.actuator_net_file.format(LEGGED_GYM_ROOT_DIR=LEGGED_GYM_ROOT_DIR))
            self.actuator_net_weights = torch.tensor(pack_lstm_weights(net), device=self.device)

    def reset_idx(self, env_ids):
        super().reset_idx(env_ids)
        self.sea_hidden_state_per_env[:, env_ids] = 0.0   # anymal.py:56-60
        self.sea_cell_state_per_env[:, env_ids] = 0.0

    def step(self, actions):
        out = super().step(actions)
        if getattr(self, "_sea_in_use", False) and not self._sea_control():
            # envs reset inside the step kernel (reset_buf) get the reset_idx zeroing of the LSTM
            # state (anymal.py:56-60); masked multiply, no host synchronisation
            keep = (~self.reset_buf).to(self.sea_hidden_state.dtype).view(1, self.num_envs, 1, 1)
            self.sea_hidden_state_per_env.mul_(keep)
            self.sea_cell_state_per_env.mul_(keep)
        return out

    def actuator_torques(self, actions):
        """anymal.py:62-78 on the lgx LSTM kernel: [N, 12] torques, hidden state advanced."""
        from legged_gym_amd.sim import lib as lgxlib
        lib = lgxlib.load()
        self._sea_in_use = True
        self.sea_input[:, 0, 0] = (actions * self.cfg.control.action_scale + self.default_dof_pos - self.dof_pos).flatten()
        self.sea_input[:, 0, 1] = self.dof_vel.flatten()
        stream = C.c_void_p(torch.cuda.current_stream(torch.device(self.device)).cuda_stream)
        lgxlib.check(lib.lgx_actuator_lstm(C.c_void_p(self.sea_input.data_ptr()), C.c_void_p(self.sea_hidden_state.data_ptr()),
                                           C.c_void_p(self.sea_cell_state.data_ptr()), C.c_void_p(self._sea_tau.data_ptr()),
                                           self._sea_tau.numel(), C.c_void_p(self.actuator_net_weights.data_ptr()), stream),
                     "lgx_actuator_lstm")
        return self._sea_tau.view(self.num_envs, self.num_actions)
