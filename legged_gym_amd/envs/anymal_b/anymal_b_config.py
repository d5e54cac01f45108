"""ANYmal-B config (reference: legged_gym/envs/anymal_b/anymal_b_config.py:33-45): the ANYmal-C
rough config with the ANYmal-B model; registered with the `Anymal` env class.
"""
from legged_gym_amd.envs.anymal_c.anymal_c_config import AnymalCRoughCfg, AnymalCRoughCfgPPO


class AnymalBRoughCfg(AnymalCRoughCfg):
    class asset(AnymalCRoughCfg.asset):
        file = "{LEGGED_GYM_ROOT_DIR}/resources/anymal_b_model.json"
        name = "anymal_b"
        foot_name = 'FOOT'


class AnymalBRoughCfgPPO(AnymalCRoughCfgPPO):
    class runner(AnymalCRoughCfgPPO.runner):
        run_name = ''
        experiment_name = 'rough_anymal_b'
        load_run = -1
