"""Extract actuator-net weights from the reference's TorchScript archives WITHOUT executing them.

`torch.load(weights_only=True)` refuses TorchScript archives and `torch.jit.load` would run
code stored in the file, so neither is used.  Instead this tool
  1. disassembles `<archive>/data.pkl` with `pickletools.genops` (a static opcode walk: nothing
     is unpickled or executed) to recover, in order, each parameter's dotted name, its storage
     key and its shape, and
  2. reads the raw little-endian float32 storage blobs `<archive>/data/<key>` with numpy.
The architecture itself (Linear/Tanh stack; LSTM + Linear with in/out scales) is read from the
archive's code text (`code/__torch__/*.py`) and from the reference's call sites
(legged_gym/envs/go1/go1.py:22-35,100-105; legged_gym/envs/anymal_c/anymal.py:62-78).

Usage: python tools/export_actuator_nets.py  (container-only; writes legged_gym_amd/resources/actuator_nets/*.npz)
"""
import os
import pickletools
import sys
import zipfile

import numpy as np

SRC = "/root/reference/resources/actuator_nets"
DST = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "legged_gym_amd", "resources",
                   "actuator_nets")


def tensors_from_archive(path, expect_names):
    """Open the archive and statically check (pickletools.genops, no execution) that the
    parameter names appear in data.pkl in the expected storage order."""
    z = zipfile.ZipFile(path)
    prefix = z.namelist()[0].split("/")[0]
    strings = [arg for op, arg, _ in pickletools.genops(z.read(prefix + "/data.pkl")) if isinstance(arg, str)]
    pos = [strings.index(n) for n in expect_names]
    assert pos == sorted(pos), f"unexpected parameter order in {path}: {pos}"
    return z, prefix, {n: p for n, p in zip(expect_names, pos)}


def raw(z, prefix, key, n):
    b = z.read(f"{prefix}/data/{key}")
    a = np.frombuffer(b, dtype="<f4")
    assert a.size == n, (key, a.size, n)
    return a.copy()


def export_go1():
    z, pre, meta = tensors_from_archive(os.path.join(SRC, "go1_net.pt"), ["architecture", "0", "2", "4", "6"])
    shapes = [(128, 30), (128,), (128, 128), (128,), (128, 128), (128,), (3, 128), (3,)]
    names = ["w0", "b0", "w1", "b1", "w2", "b2", "w3", "b3"]
    arrs = {}
    for k, (nm, sh) in enumerate(zip(names, shapes)):
        arrs[nm] = raw(z, pre, str(k), int(np.prod(sh))).reshape(sh)
    # normalisation constants of the reference wrapper (go1.py:50-53), stored alongside as data
    arrs["pos_err_mean"] = np.array([0.00036437, 0.01540757, -0.00972657], np.float32)
    arrs["pos_err_std"] = np.array([0.11722939, 0.19275887, 0.28700321], np.float32)
    arrs["vel_mean"] = np.array([-0.00017714, -0.00024455, 0.0005956], np.float32)
    arrs["vel_std"] = np.array([2.31517027, 3.84613839, 5.52599008], np.float32)
    return arrs, meta


def export_lstm():
    z, pre, meta = tensors_from_archive(os.path.join(SRC, "anydrive_v3_lstm.pt"),
                                        ["in_scale", "out_scale", "weight_ih_l0", "weight_hh_l0", "bias_ih_l0",
                                         "bias_hh_l0", "weight_ih_l1", "weight_hh_l1", "bias_ih_l1", "bias_hh_l1"])
    spec = [("in_scale", (2,)), ("out_scale", (1,)), ("w_ih_l0", (32, 2)), ("w_hh_l0", (32, 8)), ("b_ih_l0", (32,)),
            ("b_hh_l0", (32,)), ("w_ih_l1", (32, 8)), ("w_hh_l1", (32, 8)), ("b_ih_l1", (32,)), ("b_hh_l1", (32,)),
            ("w_lin", (1, 8)), ("b_lin", (1,))]
    arrs = {}
    for k, (nm, sh) in enumerate(spec):
        arrs[nm] = raw(z, pre, str(k), int(np.prod(sh))).reshape(sh)
    return arrs, meta


if __name__ == "__main__":
    os.makedirs(DST, exist_ok=True)
    g, gm = export_go1()
    np.savez(os.path.join(DST, "go1_net.npz"), **g)
    l, lm = export_lstm()
    np.savez(os.path.join(DST, "anydrive_v3_lstm.npz"), **l)
    print("go1 name order ok:", gm)
    print("lstm name order ok:", lm)
    print("in_scale", l["in_scale"], "out_scale", l["out_scale"])
    sys.exit(0)
