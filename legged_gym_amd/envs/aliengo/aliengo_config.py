"""Unitree Aliengo config (reference: legged_gym/envs/aliengo/aliengo_config.py:33-108).

Flat `plane`, 48-dim obs, Go1 gains and the Go1 actuator net (the reference points Aliengo at
go1_net.pt), base/limb mass randomisation, a 0.5 m base-height target.
"""
from legged_gym_amd.envs.base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO


class AliengoRoughCfg(LeggedRobotCfg):
    class env(LeggedRobotCfg.env):
        num_observations = 48

    class terrain(LeggedRobotCfg.terrain):
        mesh_type = 'plane'
        measure_heights = False

    class init_state(LeggedRobotCfg.init_state):
        pos = [0.0, 0.0, 0.32]
        default_joint_angles = {
            'FL_hip_joint': 0., 'RL_hip_joint': 0., 'FR_hip_joint': -0.1, 'RR_hip_joint': -0.1,
            'FL_thigh_joint': 0.6, 'RL_thigh_joint': 0.8, 'FR_thigh_joint': 0.6, 'RR_thigh_joint': 0.8,
            'FL_calf_joint': -0.7, 'RL_calf_joint': -0.7, 'FR_calf_joint': -0.7, 'RR_calf_joint': -0.7,
        }

    class control(LeggedRobotCfg.control):
        control_type = 'P'
        stiffness = {'hip_joint': 30, 'thigh_joint': 50., 'calf_joint': 50.}
        damping = {'hip_joint': 2., 'thigh_joint': 2., 'calf_joint': 2.}
        action_scale = 0.25
        decimation = 4
        use_actuator_network = True
        actuator_net_file = "{LEGGED_GYM_ROOT_DIR}/resources/actuator_nets/go1_net.npz"

    class asset(LeggedRobotCfg.asset):
        file = '{LEGGED_GYM_ROOT_DIR}/resources/aliengo_model.json'
        name = "aliengo"
        foot_name = "foot"
        penalize_contacts_on = ["thigh", "calf"]
        terminate_after_contacts_on = ["base"]
        self_collisions = 1

    class domain_rand(LeggedRobotCfg.domain_rand):
        randomize_base_mass = True
        added_mass_range = [-1., 1.]
        randomize_limb_mass = True
        added_limb_percentage = [-0.2, 0.2]

    class rewards(LeggedRobotCfg.rewards):
        soft_dof_pos_limit = 0.9
        base_height_target = 0.5

        class scales(LeggedRobotCfg.rewards.scales):
            torques = -0.00025
            dof_pos_limits = -10.0


class AliengoRoughCfgPPO(LeggedRobotCfgPPO):
    class algorithm(LeggedRobotCfgPPO.algorithm):
        entropy_coef = 0.01

    class runner(LeggedRobotCfgPPO.runner):
        run_name = ''
        experiment_name = 'rough_aliengo'
