"""The ANYmal SEA actuator network as the step's torque source (LGX_CTRL_SEA; reference
anymal.py:71-78 with use_actuator_network, reached through cfg.control.explicit_torques).

CPU: the oracle's step against torch's own nn.LSTM with the weights of the reference's
anydrive_v3_lstm.pt (extracted to resources/actuator_nets/anydrive_v3_lstm.npz): one substep
(decimation 1), so the reported torques are exactly the LSTM output of that substep; an env that
resets in the step ends it with zero LSTM state (Anymal.reset_idx, anymal.py:56-60), read back.
GPU: tests/test_gpu_parity.py::test_anymal_sea_torque_step_matches_oracle.
"""
import os

import numpy as np
import torch

from oracle_backend import make_env


def _torch_sea(net, x, h, c):
    lstm = torch.nn.LSTM(2, 8, 2)
    with torch.no_grad():
        for L in range(2):
            for k in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"):
                getattr(lstm, f"{k}_l{L}").copy_(torch.tensor(net[f"{k.replace('weight', 'w').replace('bias', 'b')}_l{L}"]))
        y, (h2, c2) = lstm((x * torch.tensor(net["in_scale"])).unsqueeze(0), (h, c))
        tau = (y[0] @ torch.tensor(net["w_lin"]).T + torch.tensor(net["b_lin"]))[:, 0] * float(net["out_scale"][0])
    return tau, h2, c2


def test_sea_torque_step_matches_torch_lstm():
    import legged_gym_amd
    from legged_gym_amd.sim.model import load_actuator_net

    def ov(c):
        c.control.explicit_torques = True
        c.control.decimation = 1
    env = make_env("anymal_c_rough", num_envs=8, device="cpu", backend="oracle", overrides=ov)
    from legged_gym_amd.sim import abi
    assert env._lgx_params.control_type == abi.CTRL["SEA"]
    net = load_actuator_net(os.path.join(legged_gym_amd.LEGGED_GYM_ROOT_DIR, "resources/actuator_nets/anydrive_v3_lstm.npz"))
    g = torch.Generator().manual_seed(3)
    N = env.num_envs
    env.dof_pos[:] = env.default_dof_pos + (torch.rand(N, 12, generator=g) - 0.5) * 0.4
    env.dof_vel[:] = (torch.rand(N, 12, generator=g) - 0.5) * 3
    env.sea_hidden_state.copy_(torch.randn(2, N * 12, 8, generator=g) * 0.3)
    env.sea_cell_state.copy_(torch.randn(2, N * 12, 8, generator=g) * 0.3)
    env._episode_length_buf[:] = torch.arange(N) * 7 + 1
    env._episode_length_buf[3] = int(env.max_episode_length)   # times out in this step
    a = (torch.rand(N, 12, generator=g) - 0.5) * 2
    x = torch.stack([(a * env.cfg.control.action_scale + env.default_dof_pos - env.dof_pos).flatten(),
                     env.dof_vel.flatten()], dim=1)
    h0, c0 = env.sea_hidden_state.clone(), env.sea_cell_state.clone()
    tau, h2, c2 = _torch_sea(net, x, h0, c0)
    env.step(a)
    assert bool(env.reset_buf[3]) and int(env.reset_buf.sum()) == 1
    h2.view(2, N, 12, 8)[:, 3] = 0      # reset_idx zeroed env 3's state after its last substep
    c2.view(2, N, 12, 8)[:, 3] = 0
    eff = env.torque_limits.repeat(N)
    want = torch.clamp(tau, -eff, eff).view(N, 12)
    assert torch.allclose(env.torques, want, atol=1e-4, rtol=1e-5), (env.torques - want).abs().max()
    assert torch.allclose(env.sea_hidden_state, h2, atol=1e-6, rtol=1e-5)
    assert torch.allclose(env.sea_cell_state, c2, atol=1e-6, rtol=1e-5)
    assert (want.abs() > 1.0).any()                      # the network actually drives the joints
