"""Unitree A1 configs: `a1` and `a1_src` (the same robot with the vendor URDF).

References: legged_gym/envs/a1/a1_config.py:33-85 and legged_gym/envs/a1_src/a1_src_config.py:34-89.
Both inherit the base terrain (plane with the 187-point height scan, 235-dim obs) and run the
plain PD drive (registered as `LeggedRobot`, envs/__init__.py:54,56); the two differ only in
the URDF and the torque penalty.
"""
from legged_gym_amd.envs.base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO


class A1RoughCfg(LeggedRobotCfg):
    class init_state(LeggedRobotCfg.init_state):
        pos = [0.0, 0.0, 0.42]
        default_joint_angles = {
            'FL_hip_joint': 0.1, 'RL_hip_joint': 0.1, 'FR_hip_joint': -0.1, 'RR_hip_joint': -0.1,
            'FL_thigh_joint': 0.8, 'RL_thigh_joint': 1., 'FR_thigh_joint': 0.8, 'RR_thigh_joint': 1.,
            'FL_calf_joint': -1.5, 'RL_calf_joint': -1.5, 'FR_calf_joint': -1.5, 'RR_calf_joint': -1.5,
        }

    class control(LeggedRobotCfg.control):
        control_type = 'P'
        stiffness = {'joint': 40.}
        damping = {'joint': 1.0}
        action_scale = 0.25
        decimation = 4

    class asset(LeggedRobotCfg.asset):
        file = '{LEGGED_GYM_ROOT_DIR}/resources/a1_model.json'
        name = "a1"
        foot_name = "foot"
        penalize_contacts_on = ["thigh", "calf"]
        terminate_after_contacts_on = ["base"]
        self_collisions = 1

    class rewards(LeggedRobotCfg.rewards):
        soft_dof_pos_limit = 0.9
        base_height_target = 0.25

        class scales(LeggedRobotCfg.rewards.scales):
            torques = -0.0002
            dof_pos_limits = -10.0


class A1RoughCfgPPO(LeggedRobotCfgPPO):
    class algorithm(LeggedRobotCfgPPO.algorithm):
        entropy_coef = 0.01

    class runner(LeggedRobotCfgPPO.runner):
        run_name = ''
        experiment_name = 'rough_a1'


class A1SrcRoughCfg(A1RoughCfg):
    class asset(A1RoughCfg.asset):
        file = '{LEGGED_GYM_ROOT_DIR}/resources/a1_src_model.json'
        name = "a1_src"

    class rewards(A1RoughCfg.rewards):
        class scales(A1RoughCfg.rewards.scales):
            torques = -0.00001


class A1SrcRoughCfgPPO(A1RoughCfgPPO):
    class runner(A1RoughCfgPPO.runner):
        experiment_name = 'rough_a1_src'
