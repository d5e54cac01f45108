"""Python shims over the PPO-side HIP kernels of liblgx.so (no fallback on GPU tensors)."""
import ctypes as C

import torch


def _vp(t):
    return C.c_void_p(t.data_ptr())


def gae(rewards, values, dones, last_values, returns, advantages, gamma, lam):
    """rewards/values/returns/advantages [T,N,1] f32, dones [T,N,1] uint8, last_values [N,1]."""
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    T, N = rewards.shape[0], rewards.shape[1]
    for t in (rewards, values, dones, returns, advantages, last_values):
        assert t.is_cuda and t.is_contiguous()
    stream = C.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    lgxlib.check(lib.lgx_gae(_vp(rewards), _vp(values), _vp(dones), _vp(last_values), _vp(returns), _vp(advantages),
                             T, N, float(gamma), float(lam), stream), "lgx_gae")


_scratch = {}


def gae_norm(rewards, values, dones, last_values, returns, advantages, gamma, lam):
    """gae() + rsl_rl's advantage normalisation in place (single process): lgx_gae_norm."""
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    T, N = rewards.shape[0], rewards.shape[1]
    for t in (rewards, values, dones, returns, advantages, last_values):
        assert t.is_cuda and t.is_contiguous()
    key = (rewards.device, N)
    if key not in _scratch:
        _scratch[key] = torch.empty(int(lib.lgx_gae_norm_scratch(N)), dtype=torch.float64, device=rewards.device)
    stream = C.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    lgxlib.check(lib.lgx_gae_norm(_vp(rewards), _vp(values), _vp(dones), _vp(last_values), _vp(returns),
                                  _vp(advantages), T, N, float(gamma), float(lam), _vp(_scratch[key]), stream),
                 "lgx_gae_norm")


def gae_parts(rewards, values, dones, last_values, returns, advantages, gamma, lam):
    """gae() + this rank's per-workgroup (count, mean, M2) advantage summaries (lgx_gae_parts):
    returns the [lgx_gae_norm_scratch(N)] float64 device tensor (data-parallel normalisation)."""
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    T, N = rewards.shape[0], rewards.shape[1]
    for t in (rewards, values, dones, returns, advantages, last_values):
        assert t.is_cuda and t.is_contiguous()
    parts = torch.empty(int(lib.lgx_gae_norm_scratch(N)), dtype=torch.float64, device=rewards.device)
    stream = C.c_void_p(torch.cuda.current_stream(rewards.device).cuda_stream)
    lgxlib.check(lib.lgx_gae_parts(_vp(rewards), _vp(values), _vp(dones), _vp(last_values), _vp(returns),
                                   _vp(advantages), T, N, float(gamma), float(lam), _vp(parts), stream),
                 "lgx_gae_parts")
    return parts


def adv_norm(advantages, parts):
    """Normalise `advantages` in place with the statistics of the (count, mean, M2) summaries
    `parts` (every rank's, in rank order): lgx_adv_norm."""
    from legged_gym_amd.sim import lib as lgxlib
    lib = lgxlib.load()
    assert advantages.is_cuda and advantages.is_contiguous() and parts.is_cuda and parts.dtype == torch.float64
    parts = parts.contiguous()
    assert parts.numel() % 3 == 0
    stream = C.c_void_p(torch.cuda.current_stream(advantages.device).cuda_stream)
    lgxlib.check(lib.lgx_adv_norm(_vp(advantages), advantages.numel(), _vp(parts), parts.numel() // 3, stream),
                 "lgx_adv_norm")
