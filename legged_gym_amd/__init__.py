"""legged_gym_amd — MI355X-native rollout engine with the legged_gym / rsl_rl surface.

LEGGED_GYM_ROOT_DIR points at this package directory (resources live under it), mirroring
legged_gym/__init__.py:33-34.
"""
import os

LEGGED_GYM_ROOT_DIR = os.path.dirname(os.path.abspath(__file__))
LEGGED_GYM_ENVS_DIR = os.path.join(LEGGED_GYM_ROOT_DIR, "envs")
