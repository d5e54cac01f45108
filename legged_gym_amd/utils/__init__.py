"""Public helpers, as `legged_gym.utils` exports them (legged_gym/utils/__init__.py)."""
from .helpers import class_to_dict, get_load_path, get_args, export_policy_as_jit, set_seed, update_class_from_dict  # noqa: F401
from .task_registry import task_registry  # noqa: F401
