"""GPU: the train / play entry points end to end (legged_gym/scripts/train.py, play.py):
2 PPO iterations with checkpointing on the HIP path, then resume the latest checkpoint,
export the actor as TorchScript and run the policy."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_then_play(gpu, tmp_path):
    from legged_gym_amd import LEGGED_GYM_ROOT_DIR
    from legged_gym_amd.scripts.play import play
    from legged_gym_amd.scripts.train import train
    from legged_gym_amd.utils import get_args
    exp = f"pytest_{os.getpid()}"
    common = ["--task", "go1", "--headless", "--num_envs", "64", "--experiment_name", exp]
    train(get_args(common + ["--max_iterations", "2"]))
    root = os.path.join(LEGGED_GYM_ROOT_DIR, "logs", exp)
    runs = os.listdir(root)
    assert len(runs) == 1 and "model_2.pt" in os.listdir(os.path.join(root, runs[0]))
    # go1_config.py pins load_run to the authors' run; point it at ours
    finished = play(get_args(common + ["--load_run", runs[0]]), steps=60)
    assert os.path.exists(os.path.join(root, "exported", "policies", "policy_1.pt"))
    pol = torch.jit.load(os.path.join(root, "exported", "policies", "policy_1.pt"))
    assert pol(torch.zeros(1, 48)).shape == (1, 12)
