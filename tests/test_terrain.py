"""Trimesh terrain with the slope correction (terrain.py:70-73: isaacgym terrain_utils
convert_heightfield_to_trimesh with cfg.slope_treshold, legged_robot_config.py:68; the mesh PhysX
collides with, legged_robot.py:629-643) and the contact model on it.

terrain_utils is absent: the vectorised restatement (utils/terrain.py) is checked against a loop
transcription of the published algorithm and against the construction's invariants, and the
contact query of the oracle against closed-form answers on a stair.  Parity with Isaac Gym /
PhysX: UNPINNED.  GPU: lgx_trimesh_build == this restatement bit for bit
(tests/test_gpu_terrain.py).
"""
import numpy as np
import pytest
import torch

from legged_gym_amd.utils.terrain import (convert_heightfield_to_trimesh, trimesh_contact_tables,
                                          trimesh_vertex_moves)


def _loop_trimesh(hf, hs, vs, slope_threshold):
    """Transcription of the published convert_heightfield_to_trimesh with its per-row triangle loop."""
    num_rows, num_cols = hf.shape
    y = np.linspace(0, (num_cols - 1) * hs, num_cols)
    x = np.linspace(0, (num_rows - 1) * hs, num_rows)
    yy, xx = np.meshgrid(y, x)
    thr = slope_threshold
    thr *= hs / vs
    h = hf.astype(np.int64)
    move_x = np.zeros((num_rows, num_cols))
    move_y = np.zeros((num_rows, num_cols))
    move_corners = np.zeros((num_rows, num_cols))
    move_x[:num_rows - 1, :] += (h[1:num_rows, :] - h[:num_rows - 1, :] > thr)
    move_x[1:num_rows, :] -= (h[:num_rows - 1, :] - h[1:num_rows, :] > thr)
    move_y[:, :num_cols - 1] += (h[:, 1:num_cols] - h[:, :num_cols - 1] > thr)
    move_y[:, 1:num_cols] -= (h[:, :num_cols - 1] - h[:, 1:num_cols] > thr)
    move_corners[:num_rows - 1, :num_cols - 1] += (h[1:num_rows, 1:num_cols] - h[:num_rows - 1, :num_cols - 1] > thr)
    move_corners[1:num_rows, 1:num_cols] -= (h[:num_rows - 1, :num_cols - 1] - h[1:num_rows, 1:num_cols] > thr)
    xx += (move_x + move_corners * (move_x == 0)) * hs
    yy += (move_y + move_corners * (move_y == 0)) * hs
    vertices = np.zeros((num_rows * num_cols, 3), dtype=np.float32)
    vertices[:, 0] = xx.flatten()
    vertices[:, 1] = yy.flatten()
    vertices[:, 2] = hf.flatten() * vs
    triangles = -np.ones((2 * (num_rows - 1) * (num_cols - 1), 3), dtype=np.uint32)
    for i in range(num_rows - 1):
        ind0 = np.arange(0, num_cols - 1) + i * num_cols
        ind1 = ind0 + 1
        ind2 = ind0 + num_cols
        ind3 = ind2 + 1
        start = 2 * i * (num_cols - 1)
        stop = start + 2 * (num_cols - 1)
        triangles[start:stop:2, 0] = ind0
        triangles[start:stop:2, 1] = ind3
        triangles[start:stop:2, 2] = ind1
        triangles[start + 1:stop:2, 0] = ind0
        triangles[start + 1:stop:2, 1] = ind2
        triangles[start + 1:stop:2, 2] = ind3
    return vertices, triangles


def _stairs(rows=40, cols=30, step=30, width=3):
    hf = np.zeros((rows, cols), np.int16)
    for i in range(rows):
        hf[i, :] = (i // width) * step          # risers between rows 3k-1 and 3k, 0.15 m at vs 0.005
    hf[:, 20:] = 0                              # a cliff along y too (corner moves)
    return hf


def test_vectorised_trimesh_equals_loop_transcription():
    rng = np.random.default_rng(0)
    for hf in (_stairs(), rng.integers(-40, 40, size=(31, 27)).astype(np.int16)):
        v, t = convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
        v2, t2 = _loop_trimesh(hf, 0.1, 0.005, 0.75)
        np.testing.assert_array_equal(v, v2)
        np.testing.assert_array_equal(t, t2)
        v0, _ = convert_heightfield_to_trimesh(hf, 0.1, 0.005, None)   # no correction: the plain grid
        np.testing.assert_array_equal(v0[:, :2].reshape(*hf.shape, 2)[:, 0, 0], np.linspace(0, 0.1 * (hf.shape[0] - 1),
                                                                                            hf.shape[0]).astype(np.float32))


def test_slope_correction_makes_risers_vertical():
    hf = _stairs()
    dx, dy = trimesh_vertex_moves(hf, 0.1, 0.005, 0.75)
    v, _ = convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    V = v.reshape(*hf.shape, 3)
    # a riser: rows 2 -> 3 rise by 30 units > 15 = 0.75 * 0.1 / 0.005: the lower row moves onto the
    # upper row's x, so the two rows form a vertical face
    for j in range(0, 19):
        assert dx[2, j] == 1 and V[2, j, 0] == V[3, j, 0] and V[2, j, 2] < V[3, j, 2]
        assert dx[1, j] == 0 and dx[3, j] == 0
    # gentle slopes (below the threshold) are left alone
    gentle = (np.arange(40)[:, None] * 10 + np.zeros((1, 30))).astype(np.int16)
    gx, gy = trimesh_vertex_moves(gentle, 0.1, 0.005, 0.75)
    assert not gx.any() and not gy.any()
    # the cliff along y at col 20 (higher side cols < 20): the lower column moves toward it
    assert (dy[3:, 20] == -1).all()
    code, flag = trimesh_contact_tables(dx, dy)
    assert code.min() >= 0 and code.max() <= 8 and (code[dx == 0] % 3 == dy[dx == 0] + 1).all()
    moved = (dx != 0) | (dy != 0)
    for i, j in [(2, 5), (0, 0), (10, 10), (39, 29), (20, 19)]:
        want = moved[max(i - 1, 0):i + 3, max(j - 1, 0):j + 3].any()
        assert bool(flag[i, j]) == want, (i, j)


def _stair_env():
    """A 64-env oracle env whose heightfield is replaced by the stair of _stairs (border 0)."""
    from oracle_backend import make_env

    def ov(c):
        c.terrain.border_size = 0.0
    env = make_env("go1_rough", num_envs=8, device="cpu", backend="oracle", overrides=ov)
    hf = np.zeros(tuple(env.height_samples.shape), np.int16)
    hf[:40, :30] = _stairs()
    env.height_samples.copy_(torch.from_numpy(hf))
    env.hf_trimesh.copy_(env._trimesh_contact_table())
    return env


def _contact(env, p, r):
    import ctypes as C
    from oracle_backend import load_oracle
    n = torch.zeros(3)
    pt = torch.tensor(p, dtype=torch.float32)
    d = load_oracle().lgxo_ground_contact(C.byref(env._lgx_params), C.byref(env._lgx_bufs), C.c_void_p(pt.data_ptr()),
                                          r, C.c_void_p(n.data_ptr()))
    return d, n.numpy()


def test_contact_on_the_corrected_stair():
    env = _stair_env()
    if env.cfg.terrain.border_size != 0.0:
        pytest.skip("border override not applied")
    r = 0.02
    # the riser between rows 2 and 3 is the vertical face x = 0.3 from z = 0 to z = 0.15
    d, n = _contact(env, (0.29, 0.5, 0.05), r)            # beside the face, lower side, 1 cm away
    assert d == pytest.approx(r - 0.01, abs=1e-5) and n == pytest.approx([-1, 0, 0], abs=1e-5)
    d, n = _contact(env, (0.25, 0.5, 0.05), r)            # 5 cm away: no contact (depth < 0; the
    assert d < 0                                          # cells farther than r are culled)
    d, n = _contact(env, (0.285, 0.5, 0.05), r)           # 1.5 cm away, still within r: contact
    assert d == pytest.approx(r - 0.015, abs=1e-5) and n == pytest.approx([-1, 0, 0], abs=1e-5)
    d, n = _contact(env, (0.45, 0.5, 0.16), r)            # above the upper tread, 1 cm up
    assert d == pytest.approx(r - 0.01, abs=1e-5) and n == pytest.approx([0, 0, 1], abs=1e-5)
    d, n = _contact(env, (0.45, 0.5, 0.145), r)           # 5 mm into the tread
    assert d == pytest.approx(r + 0.005, abs=1e-5) and n == pytest.approx([0, 0, 1], abs=1e-5)
    d, n = _contact(env, (0.302, 0.5, 0.10), r)           # inside the step, 2 mm behind the face
    assert d == pytest.approx(r + 0.002, abs=1e-5) and n == pytest.approx([-1, 0, 0], abs=1e-5)
    # box corners (radius 0) query the heightfield triangle under them, even beside the riser:
    # 0.1 cm from the face, on the raw ramp of cell row 2 (0 -> 0.15 m over x 0.2 .. 0.3)
    d, n = _contact(env, (0.299, 0.5, 0.05), 0.0)
    assert d == pytest.approx((0.15 * 0.99 - 0.05) / np.sqrt(1 + 1.5 ** 2), abs=1e-5)
    # far from any moved vertex: the heightfield query (identical surface), e.g. the flat ground
    # beyond the stair
    d, n = _contact(env, (2.0, 2.5, 0.01), r)
    assert d == pytest.approx(r - 0.01, abs=1e-6) and n == pytest.approx([0, 0, 1], abs=1e-6)
