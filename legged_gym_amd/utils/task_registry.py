"""Task registry: name -> (env class, env cfg, train cfg); env and runner factories.

Same API and behaviour as legged_gym/utils/task_registry.py:46-171 (register / get_task_class /
get_cfgs / make_env / make_alg_runner, log-dir layout and resume).  The runner is the in-repo
rsl_rl-compatible `OnPolicyRunner` (legged_gym_amd.rl) unless `rsl_rl` is importable and
`LGX_USE_RSL_RL=1` is set, in which case the upstream runner drops in unchanged.
"""
import os
import shutil
from datetime import datetime
from typing import TYPE_CHECKING, Tuple

from legged_gym_amd import LEGGED_GYM_ROOT_DIR

if TYPE_CHECKING:  # avoid the envs/__init__ -> task_registry import cycle
    from legged_gym_amd.envs.base.legged_robot_config import LeggedRobotCfg, LeggedRobotCfgPPO

from .helpers import class_to_dict, get_args, get_load_path, parse_sim_params, set_seed, update_cfg_from_args


def _runner_class():
    if os.environ.get("LGX_USE_RSL_RL") == "1":
        from rsl_rl.runners import OnPolicyRunner  # noqa: the upstream runner, if installed
        return OnPolicyRunner
    from legged_gym_amd.rl.runner import OnPolicyRunner
    return OnPolicyRunner


class TaskRegistry:
    def __init__(self):
        self.task_classes = {}
        self.env_cfgs = {}
        self.train_cfgs = {}

    def register(self, name: str, task_class, env_cfg: "LeggedRobotCfg", train_cfg: "LeggedRobotCfgPPO"):
        self.task_classes[name] = task_class
        self.env_cfgs[name] = env_cfg
        self.train_cfgs[name] = train_cfg

    def get_task_class(self, name: str):
        return self.task_classes[name]

    def get_cfgs(self, name) -> Tuple["LeggedRobotCfg", "LeggedRobotCfgPPO"]:
        train_cfg = self.train_cfgs[name]
        env_cfg = self.env_cfgs[name]
        env_cfg.seed = train_cfg.seed  # task_registry.py:63-64
        return env_cfg, train_cfg

    def make_env(self, name, args=None, env_cfg=None):
        if args is None:
            args = get_args()
        if name not in self.task_classes:
            raise ValueError(f"Task with name: {name} was not registered")
        task_class = self.get_task_class(name)
        if env_cfg is None:
            env_cfg, _ = self.get_cfgs(name)
        env_cfg, _ = update_cfg_from_args(env_cfg, None, args)
        if not hasattr(env_cfg, "seed"):  # a fresh cfg instance: seed from the registered train cfg
            env_cfg.seed = self.train_cfgs[name].seed
        set_seed(env_cfg.seed)
        sim_params = parse_sim_params(args, {"sim": class_to_dict(env_cfg.sim)})
        env = task_class(cfg=env_cfg, sim_params=sim_params, physics_engine=args.physics_engine,
                         sim_device=args.sim_device, headless=args.headless)
        return env, env_cfg

    def make_alg_runner(self, env, name=None, args=None, train_cfg=None, log_root="default"):
        if args is None:
            args = get_args()
        if train_cfg is None:
            if name is None:
                raise ValueError("Either 'name' or 'train_cfg' must be not None")
            _, train_cfg = self.get_cfgs(name)
        elif name is not None:
            print(f"'train_cfg' provided -> Ignoring 'name={name}'")
        _, train_cfg = update_cfg_from_args(None, train_cfg, args)
        stamp = datetime.now().strftime("%b%d_%H-%M-%S") + "_" + train_cfg.runner.run_name
        if log_root == "default":
            log_root = os.path.join(LEGGED_GYM_ROOT_DIR, "logs", train_cfg.runner.experiment_name)
            log_dir = os.path.join(log_root, stamp)
        elif log_root is None:
            log_dir = None
        else:
            log_dir = os.path.join(log_root, stamp)
        if log_dir is not None and not train_cfg.runner.resume:
            os.makedirs(log_dir, exist_ok=True)
            # config snapshot (task_registry.py:148-155); folder lookup fixed for anymal_c_* tasks
            base = os.path.join(LEGGED_GYM_ROOT_DIR, "envs", "base", "legged_robot_config.py")
            shutil.copyfile(base, os.path.join(log_dir, "train_cfg_general.py"))
            if name is not None:
                folder = name.split("_")[0] if not os.path.isdir(os.path.join(LEGGED_GYM_ROOT_DIR, "envs", name)) else name
                for cand in (os.path.join(LEGGED_GYM_ROOT_DIR, "envs", folder, folder + "_config.py"),
                             os.path.join(LEGGED_GYM_ROOT_DIR, "envs", "anymal_c", "anymal_c_config.py")):
                    if os.path.exists(cand):
                        shutil.copyfile(cand, os.path.join(log_dir, "train_cfg_robot.py"))
                        break
        runner = _runner_class()(env, class_to_dict(train_cfg), log_dir, device=args.rl_device)
        if train_cfg.runner.resume:
            resume_path = get_load_path(log_root, load_run=train_cfg.runner.load_run,
                                        checkpoint=train_cfg.runner.checkpoint)
            print(f"Loading model from: {resume_path}")
            runner.load(resume_path)
        return runner, train_cfg


task_registry = TaskRegistry()
