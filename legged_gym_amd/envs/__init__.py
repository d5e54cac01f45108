"""Task registrations (legged_gym/envs/__init__.py:52-59) for the robots in BASELINE scope.

go1 (configs C1/C2 defaults), go1_rough (C3/C4: trimesh + height scan), go1_flat_bench (C2 as
BASELINE states it: PD, no domain randomisation), anymal_c_rough (C5), anymal_c_flat.
"""
from legged_gym_amd import LEGGED_GYM_ENVS_DIR, LEGGED_GYM_ROOT_DIR  # noqa: F401
from legged_gym_amd.utils.task_registry import task_registry

from .anymal_c.anymal import Anymal
from .anymal_c.anymal_c_config import AnymalCFlatCfg, AnymalCFlatCfgPPO, AnymalCRoughCfg, AnymalCRoughCfgPPO
from .base.legged_robot import LeggedRobot
from .base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO
from .go1.go1 import Go1
from .go1.go1_config import Go1FlatBenchCfg, Go1RoughCfg, Go1RoughCfgPPO, Go1RoughTerrainCfg

task_registry.register("go1", Go1, Go1RoughCfg(), Go1RoughCfgPPO())
task_registry.register("go1_flat_bench", Go1, Go1FlatBenchCfg(), Go1RoughCfgPPO())
task_registry.register("go1_rough", Go1, Go1RoughTerrainCfg(), Go1RoughCfgPPO())
task_registry.register("anymal_c_rough", Anymal, AnymalCRoughCfg(), AnymalCRoughCfgPPO())
task_registry.register("anymal_c_flat", Anymal, AnymalCFlatCfg(), AnymalCFlatCfgPPO())
