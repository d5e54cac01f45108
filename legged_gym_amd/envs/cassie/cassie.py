"""Cassie env (reference: legged_gym/envs/cassie/cassie.py:41-46).

The reference adds one reward term to LeggedRobot, `_reward_no_fly`: 1 when exactly one foot has a
vertical contact force above 0.1 N.  Here it is reward term LGX_R_NO_FLY of the post-physics kernel
(lgx_envlogic.hip; the oracle restates it) - the class only exists so the registry, configs and
checkpoints name the robot as the reference does.  The biped's 2 legs x 6 joints run on the dense
joint-space physics kernel (lgx_physics_dense_kernel: lgx_model.leg_dof = 6), the quadrupeds' on the
arrowhead kernel.
"""
from legged_gym_amd.envs.base.legged_robot import LeggedRobot


class Cassie(LeggedRobot):
    pass
