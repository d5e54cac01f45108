"""Task registrations (legged_gym/envs/__init__.py:52-59) for the robots in BASELINE scope.

go1 (configs C1/C2 defaults), go1_rough (C3/C4: trimesh + height scan), go1_flat_bench (C2 as
BASELINE states it: PD, no domain randomisation), anymal_c_rough (C5), anymal_c_flat, and the
remaining robots of the reference registry: anymal_b, a1, a1_src, aliengo and cassie (the biped:
2 legs x 6 joints on the dense physics kernel).
"""
from legged_gym_amd import LEGGED_GYM_ENVS_DIR, LEGGED_GYM_ROOT_DIR  # noqa: F401
from legged_gym_amd.utils.task_registry import task_registry

from .a1.a1_config import A1RoughCfg, A1RoughCfgPPO, A1SrcRoughCfg, A1SrcRoughCfgPPO
from .aliengo.aliengo import Aliengo
from .aliengo.aliengo_config import AliengoRoughCfg, AliengoRoughCfgPPO
from .anymal_b.anymal_b_config import AnymalBRoughCfg, AnymalBRoughCfgPPO
from .anymal_c.anymal import Anymal
from .anymal_c.anymal_c_config import AnymalCFlatCfg, AnymalCFlatCfgPPO, AnymalCRoughCfg, AnymalCRoughCfgPPO
from .base.legged_robot import LeggedRobot
from .cassie.cassie import Cassie
from .cassie.cassie_config import CassieRoughCfg, CassieRoughCfgPPO
from .base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO
from .go1.go1 import Go1
from .go1.go1_config import Go1FlatBenchCfg, Go1RoughCfg, Go1RoughCfgPPO, Go1RoughTerrainCfg

task_registry.register("go1", Go1, Go1RoughCfg(), Go1RoughCfgPPO())
task_registry.register("go1_flat_bench", Go1, Go1FlatBenchCfg(), Go1RoughCfgPPO())
task_registry.register("go1_rough", Go1, Go1RoughTerrainCfg(), Go1RoughCfgPPO())
task_registry.register("anymal_c_rough", Anymal, AnymalCRoughCfg(), AnymalCRoughCfgPPO())
task_registry.register("anymal_c_flat", Anymal, AnymalCFlatCfg(), AnymalCFlatCfgPPO())
task_registry.register("anymal_b", Anymal, AnymalBRoughCfg(), AnymalBRoughCfgPPO())
task_registry.register("a1", LeggedRobot, A1RoughCfg(), A1RoughCfgPPO())
task_registry.register("a1_src", LeggedRobot, A1SrcRoughCfg(), A1SrcRoughCfgPPO())
task_registry.register("aliengo", Aliengo, AliengoRoughCfg(), AliengoRoughCfgPPO())
task_registry.register("cassie", Cassie, CassieRoughCfg(), CassieRoughCfgPPO())
