"""Config base class: nested config classes are instantiated recursively on construction.

Mirrors the reference contract of `BaseConfig.__init__` / `init_member_classes`
(legged_gym/envs/base/base_config.py:33-55): every attribute reachable through `dir()` that
is a class (except `__class__`) is replaced by an instance of itself, depth first, so that
`cfg.env.num_envs = 8` mutates only that config object.
"""
import inspect


class BaseConfig:
    def __init__(self) -> None:
        self.init_member_classes(self)

    @staticmethod
    def init_member_classes(obj):
        for name in dir(obj):
            if name == "__class__":
                continue
            member = getattr(obj, name)
            if inspect.isclass(member):
                instance = member()
                setattr(obj, name, instance)
                BaseConfig.init_member_classes(instance)
