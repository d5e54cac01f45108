"""Aliengo env (legged_gym/envs/aliengo/aliengo.py:37-107).

The reference class is the Go1 class under another name: same 5-deep actuator history, same
go1_net normalisation constants (aliengo.py:50-53 equal go1.py:50-53), same discarded dVel.
It therefore shares the Go1 implementation (history fused into the physics kernel, MLP on
f32 MFMA); only the config differs.
"""
from legged_gym_amd.envs.go1.go1 import Go1


class Aliengo(Go1):
    pass
