"""CPU tests of the boundary: C-ABI symbols/layout, config semantics, registry, host helpers.
No compute call reaches liblgx.so here (no GPU in the test container)."""
import ctypes as C
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "lgx.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lgx_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_abi():
    fns = header_functions()
    from legged_gym_amd.sim import abi
    assert sorted(abi.EXPORTED) == fns


def test_library_loads_and_exports_every_symbol():
    path = os.path.join(ROOT, "legged_gym_amd", "liblgx.so")
    assert os.path.exists(path), "run __graft_entry__.build() first"
    import torch  # noqa: F401  (HIP runtime first)
    lib = C.CDLL(path)
    for fn in header_functions():
        assert hasattr(lib, fn), fn
    from legged_gym_amd.sim import abi
    abi.declare(lib)
    abi.check_layout(lib.lgx_struct_sizes)
    assert lib.lgx_version() == 1


def test_comm_entry_points_validate_without_a_gpu():
    """lgx_comm_* / lgx_allreduce_grads argument and library checks (host-side only: no RCCL call
    and no device is reached)."""
    import torch  # noqa: F401
    from legged_gym_amd.sim import abi
    lib = abi.declare(C.CDLL(os.path.join(ROOT, "legged_gym_amd", "liblgx.so")))
    uid = (C.c_uint8 * 128)()
    assert lib.lgx_comm_unique_id(b"/nonexistent/librccl.so", uid) == -1
    assert b"not loadable" in lib.lgx_last_error()
    comm = C.c_void_p()
    assert lib.lgx_comm_create(None, uid, 2, 2, 0, C.byref(comm)) == -1      # rank >= nranks
    assert lib.lgx_comm_create(None, None, 1, 0, 0, C.byref(comm)) == -1     # no id
    assert lib.lgx_allreduce_grads(None, None, 4, 0, None) == -1
    assert lib.lgx_comm_destroy(None) == 0


def test_native_allreduce_refuses_to_fall_back(monkeypatch):
    """LGX_NATIVE_ALLREDUCE=1 on a process group that is not RCCL raises instead of silently using
    torch.distributed; unset, the torch path is taken (no communicator)."""
    import pytest
    from legged_gym_amd.rl.fused_ppo import FusedPPOUpdate

    class Dist:
        @staticmethod
        def get_backend():
            return "gloo"

    class Ppo:
        dist = Dist()
    f = FusedPPOUpdate.__new__(FusedPPOUpdate)
    f.ppo = Ppo()
    monkeypatch.delenv("LGX_NATIVE_ALLREDUCE", raising=False)
    assert f._lgx_comm() is None and f.allreduce_impl == "torch"
    f = FusedPPOUpdate.__new__(FusedPPOUpdate)
    f.ppo = Ppo()
    monkeypatch.setenv("LGX_NATIVE_ALLREDUCE", "1")
    with pytest.raises(RuntimeError, match="nccl"):
        f._lgx_comm()


def test_oracle_layout_matches():
    from oracle_backend import load_oracle
    load_oracle()  # check_layout inside


def test_class_to_dict_is_alphabetical_and_recursive():
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfg
    from legged_gym_amd.utils.helpers import class_to_dict
    d = class_to_dict(Go1RoughCfg.rewards.scales)
    assert list(d) == sorted(d)
    nz = [k for k, v in d.items() if v != 0]
    assert nz == ["action_rate", "ang_vel_xy", "collision", "dof_acc", "dof_pos_limits", "feet_air_time",
                  "lin_vel_z", "torques", "tracking_ang_vel", "tracking_lin_vel"]
    cfg = Go1RoughCfg()
    assert isinstance(class_to_dict(cfg)["sim"]["physx"], dict)


def test_base_config_instantiates_nested_classes():
    from legged_gym_amd.envs.go1.go1_config import Go1RoughCfg
    a, b = Go1RoughCfg(), Go1RoughCfg()
    a.env.num_envs = 3
    assert b.env.num_envs == 4096 and not isinstance(a.env, type)


def test_update_class_from_dict_roundtrip():
    from legged_gym_amd.envs.base.legged_robot_config import LeggedRobotCfgPPO
    from legged_gym_amd.utils.helpers import class_to_dict, update_class_from_dict
    class Cfg(LeggedRobotCfgPPO):   # helpers.py:58-65 recurses into nested config *classes*
        class runner(LeggedRobotCfgPPO.runner):
            pass
    update_class_from_dict(Cfg, {"runner": {"max_iterations": 7}, "seed": 3})
    cfg = Cfg()
    assert cfg.runner.max_iterations == 7 and cfg.seed == 3
    assert class_to_dict(cfg)["algorithm"]["num_mini_batches"] == 4


def test_registry_and_cli_overrides():
    import legged_gym_amd.envs  # noqa: F401
    from legged_gym_amd.utils.helpers import get_args, update_cfg_from_args
    from legged_gym_amd.utils.task_registry import task_registry
    assert {"go1", "go1_rough", "go1_flat_bench", "anymal_c_rough", "anymal_c_flat"} <= set(task_registry.task_classes)
    env_cfg, train_cfg = task_registry.get_cfgs("go1")
    assert env_cfg.seed == train_cfg.seed == 1
    args = get_args(["--task", "go1", "--num_envs", "17", "--seed", "5", "--max_iterations", "3", "--sim_device", "cpu"])
    e, t = update_cfg_from_args(type(env_cfg)(), type(train_cfg)(), args)
    assert e.env.num_envs == 17 and t.seed == 5 and t.runner.max_iterations == 3
    assert args.sim_device == "cpu" and args.rl_device == "cuda:0"


def test_get_load_path(tmp_path):
    from legged_gym_amd.utils.helpers import get_load_path
    for run in ["Jan01_00-00-00_a", "Feb02_00-00-00_b"]:
        (tmp_path / run).mkdir()
        for it in [0, 50, 100]:
            (tmp_path / run / f"model_{it}.pt").write_text("x")
    p = get_load_path(str(tmp_path))
    assert p.endswith(os.path.join("Jan01_00-00-00_a", "model_100.pt"))  # lexicographic run order, as the reference
    assert get_load_path(str(tmp_path), load_run="Feb02_00-00-00_b", checkpoint=50).endswith("model_50.pt")


def test_env_requires_gpu_backend_on_cpu_device():
    """The product backend fails loudly without a GPU (no CPU fallback)."""
    import legged_gym_amd.envs  # noqa: F401
    from legged_gym_amd.sim.lib import LgxError
    from legged_gym_amd.utils.helpers import get_args
    from legged_gym_amd.utils.task_registry import task_registry
    env_cfg, _ = task_registry.get_cfgs("go1_flat_bench")
    cfg = type(env_cfg)()
    cfg.env.num_envs = 4
    with pytest.raises(LgxError):
        task_registry.make_env("go1_flat_bench", args=get_args(["--sim_device", "cpu"]), env_cfg=cfg)


def test_robot_models_from_urdf():
    from legged_gym_amd.sim.model import RobotAsset
    import legged_gym_amd
    go1 = RobotAsset(os.path.join(legged_gym_amd.LEGGED_GYM_ROOT_DIR, "resources", "go1_model.json"))
    assert go1.body_names[:5] == ["base", "FL_hip", "FL_thigh", "FL_calf", "FL_foot"]
    assert go1.find_bodies("foot") == [4, 8, 12, 16]
    assert go1.dof_names[0::3] == ["FL_hip_joint", "FR_hip_joint", "RL_hip_joint", "RR_hip_joint"]
    assert abs(go1.nominal_mass.sum() - 12.01308) < 1e-4     # go1.urdf link masses
    assert go1.dof_effort.tolist() == [23.7] * 12
    an = RobotAsset(os.path.join(legged_gym_amd.LEGGED_GYM_ROOT_DIR, "resources", "anymal_c_model.json"))
    assert an.find_bodies("FOOT") == [4, 8, 12, 16] and an.dof_names[:3] == ["LF_HAA", "LF_HFE", "LF_KFE"]


def test_terrain_generator_shapes():
    from legged_gym_amd.envs.go1.go1_config import Go1RoughTerrainCfg
    from legged_gym_amd.utils.terrain import Terrain
    np.random.seed(0)
    t = Terrain(Go1RoughTerrainCfg().terrain, 64)
    assert t.heightsamples.shape == (1300, 2100) and t.heightsamples.dtype == np.int16
    assert t.env_origins.shape == (10, 20, 3)
    assert np.allclose(t.env_origins[3, 7, :2], [(3 + .5) * 8, (7 + .5) * 8])


def test_philox_stream_is_uniform_and_deterministic():
    from oracle_backend import load_oracle
    lib = load_oracle()
    u = np.array([lib.lgxo_uniform(1, e, s, 5, 0) for e in range(64) for s in range(64)])
    assert 0 <= u.min() and u.max() < 1 and abs(u.mean() - 0.5) < 0.02
    assert lib.lgxo_uniform(1, 3, 7, 5, 0) == lib.lgxo_uniform(1, 3, 7, 5, 0)
    assert lib.lgxo_uniform(1, 3, 7, 5, 0) != lib.lgxo_uniform(1, 3, 7, 6, 0)


@pytest.mark.parametrize("robot", ["go1", "cassie"])
@pytest.mark.parametrize("field,value,msg", [("point_dyn", 13, "point_dyn"), ("point_dyn", -1, "point_dyn"),
                                             ("point_report", 17, "point_report")])
def test_sim_create_rejects_bad_contact_tables(robot, field, value, msg):
    """lgx_sim_create validates every contact candidate's dyn / report body index for BOTH physics
    kernels (the dense kernel's path skipped the check and would read LDS out of bounds).
    The validation precedes any device call, so it runs here without a GPU."""
    import types
    from legged_gym_amd.sim import abi
    from legged_gym_amd.sim.model import RobotAsset, build_model
    from legged_gym_amd.utils.task_registry import task_registry
    import legged_gym_amd.envs  # noqa: F401
    task = {"go1": "go1_flat_bench", "cassie": "cassie"}[robot]
    env_cfg, _ = task_registry.get_cfgs(task)
    asset = RobotAsset(os.path.join(ROOT, "legged_gym_amd", "resources", f"{robot}_model.json"))
    model = build_model(asset, env_cfg, types.SimpleNamespace(gravity=[0.0, 0.0, -9.81], dt=0.005))
    getattr(model, field)[model.num_points - 1] = value
    p = abi.LgxEnvParams()
    p.num_envs, p.num_obs, p.decimation, p.resample_interval = 16, 48, 4, 100
    b = abi.LgxBuffers()
    for name, typ in b._fields_:
        if typ is C.c_void_p or (isinstance(typ, type) and issubclass(typ, C._Pointer)):
            setattr(b, name, C.cast(C.c_void_p(0x1000), typ) if typ is not C.c_void_p else 0x1000)
    import torch  # noqa: F401  (HIP runtime first)
    lib = C.CDLL(os.path.join(ROOT, "legged_gym_amd", "liblgx.so"))
    abi.declare(lib)
    h = C.c_void_p()
    rc = lib.lgx_sim_create(C.byref(model), C.byref(p), C.byref(b), 0, C.byref(h))
    assert rc == -1 and not h.value
    assert msg in lib.lgx_last_error().decode()
