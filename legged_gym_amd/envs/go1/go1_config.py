"""Go1 task configs (reference: legged_gym/envs/go1/go1_config.py:34-110).

`Go1RoughCfg` is the reference's Go1 config (despite the name: flat `plane`, 48-dim obs).
`Go1RoughTerrainCfg` is BASELINE config C3/C4: the same robot on the curriculum trimesh
with the 187-point height scan (235-dim obs), as SURVEY.md §8 defines it.
"""
from legged_gym_amd.envs.base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO


class Go1RoughCfg(LeggedRobotCfg):
    class env(LeggedRobotCfg.env):
        num_observations = 48

    class terrain(LeggedRobotCfg.terrain):
        mesh_type = 'plane'
        measure_heights = False

    class init_state(LeggedRobotCfg.init_state):
        pos = [0.0, 0.0, 0.32]
        default_joint_angles = {   # target angles [rad] for action = 0
            'FL_hip_joint': 0.1, 'RL_hip_joint': 0.1, 'FR_hip_joint': -0.1, 'RR_hip_joint': -0.1,
            'FL_thigh_joint': 0.8, 'RL_thigh_joint': 1., 'FR_thigh_joint': 0.8, 'RR_thigh_joint': 1.,
            'FL_calf_joint': -1.5, 'RL_calf_joint': -1.5, 'FR_calf_joint': -1.5, 'RR_calf_joint': -1.5,
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
        file = '{LEGGED_GYM_ROOT_DIR}/resources/go1_model.json'
        name = "go1"
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
        base_height_target = 0.25

        class scales(LeggedRobotCfg.rewards.scales):
            torques = -0.00025
            dof_pos_limits = -10.0


class Go1RoughCfgPPO(LeggedRobotCfgPPO):
    class algorithm(LeggedRobotCfgPPO.algorithm):
        entropy_coef = 0.01

    class runner(LeggedRobotCfgPPO.runner):
        run_name = ''
        experiment_name = 'rough_go1'


class Go1FlatBenchCfg(Go1RoughCfg):
    """BASELINE config C2: flat, PD actuator, no domain randomisation."""
    class control(Go1RoughCfg.control):
        use_actuator_network = False

    class domain_rand(Go1RoughCfg.domain_rand):
        randomize_friction = False
        randomize_base_mass = False
        randomize_limb_mass = False
        push_robots = False


class Go1RoughTerrainCfg(Go1RoughCfg):
    """BASELINE config C3/C4: curriculum trimesh + 187-point height scan, actuator net on."""
    class env(Go1RoughCfg.env):
        num_observations = 235

    class terrain(Go1RoughCfg.terrain):
        mesh_type = 'trimesh'
        measure_heights = True
