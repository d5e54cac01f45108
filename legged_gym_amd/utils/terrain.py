"""Procedural curriculum terrain (setup-time, numpy).

Mirrors legged_gym/utils/terrain.py:38-187 (Terrain: curriculum / randomized / selected maps,
sub-terrain placement, env origins, gap and pit terrains).  The sub-terrain primitives of the
un-vendored `isaacgym.terrain_utils` (pyramid slopes, random uniform noise, stairs, discrete
obstacles, stepping stones) are restated here from their published behaviour: parity with
Isaac Gym's generator is UNPINNED (the library is absent; its random_uniform_terrain also
depends on scipy.interpolate.interp2d, removed in the installed scipy).  The kernels consume
only the resulting int16 heightfield, so height-scan parity tests feed the same array to the
oracle and the kernel.
"""
import numpy as np
from scipy.interpolate import RegularGridInterpolator


class SubTerrain:
    def __init__(self, width, length, vertical_scale, horizontal_scale):
        self.width = width
        self.length = length
        self.vertical_scale = vertical_scale
        self.horizontal_scale = horizontal_scale
        self.height_field_raw = np.zeros((width, length), dtype=np.int16)


def _platform_window(t, platform_size):
    half = int(platform_size / t.horizontal_scale / 2)
    return t.width // 2 - half, t.width // 2 + half, t.length // 2 - half, t.length // 2 + half


def pyramid_sloped_terrain(t, slope=1.0, platform_size=1.0):
    cx, cy = t.width // 2, t.length // 2
    fx = (cx - np.abs(cx - np.arange(t.width))) / cx
    fy = (cy - np.abs(cy - np.arange(t.length))) / cy
    peak = int(slope * (t.horizontal_scale / t.vertical_scale) * (t.width / 2))
    t.height_field_raw += (peak * fx[:, None] * fy[None, :]).astype(np.int16)
    x1, _, y1, _ = _platform_window(t, platform_size)
    h = t.height_field_raw[x1, y1]
    t.height_field_raw = np.clip(t.height_field_raw, min(h, 0), max(h, 0))
    return t


def random_uniform_terrain(t, min_height, max_height, step=1.0, downsampled_scale=None):
    if downsampled_scale is None:
        downsampled_scale = t.horizontal_scale
    lo, hi, st = int(min_height / t.vertical_scale), int(max_height / t.vertical_scale), int(step / t.vertical_scale)
    levels = np.arange(lo, hi + st, st)
    nx = int(t.width * t.horizontal_scale / downsampled_scale)
    ny = int(t.length * t.horizontal_scale / downsampled_scale)
    coarse = np.random.choice(levels, (nx, ny))
    gx = np.linspace(0, t.width * t.horizontal_scale, nx)
    gy = np.linspace(0, t.length * t.horizontal_scale, ny)
    f = RegularGridInterpolator((gx, gy), coarse.astype(np.float64), method="linear")
    fx = np.linspace(0, t.width * t.horizontal_scale, t.width)
    fy = np.linspace(0, t.length * t.horizontal_scale, t.length)
    X, Y = np.meshgrid(fx, fy, indexing="ij")
    t.height_field_raw += np.rint(f(np.stack([X, Y], -1))).astype(np.int16)
    return t


def pyramid_stairs_terrain(t, step_width, step_height, platform_size=1.0):
    sw = int(step_width / t.horizontal_scale)
    sh = int(step_height / t.vertical_scale)
    plat = int(platform_size / t.horizontal_scale)
    h = 0
    x0, x1, y0, y1 = 0, t.width, 0, t.length
    while (x1 - x0) > plat and (y1 - y0) > plat:
        x0 += sw; x1 -= sw; y0 += sw; y1 -= sw
        h += sh
        t.height_field_raw[x0:x1, y0:y1] = h
    return t


def discrete_obstacles_terrain(t, max_height, min_size, max_size, num_rects, platform_size=1.0):
    mh = int(max_height / t.vertical_scale)
    smin, smax = int(min_size / t.horizontal_scale), int(max_size / t.horizontal_scale)
    plat = int(platform_size / t.horizontal_scale)
    heights = [-mh, -mh // 2, mh // 2, mh]
    for _ in range(num_rects):
        w = np.random.choice(range(smin, smax, 4))
        l = np.random.choice(range(smin, smax, 4))
        sx = np.random.choice(range(0, t.width - w, 4))
        sy = np.random.choice(range(0, t.length - l, 4))
        t.height_field_raw[sx:sx + w, sy:sy + l] = np.random.choice(heights)
    x1, x2 = (t.width - plat) // 2, (t.width + plat) // 2
    y1, y2 = (t.length - plat) // 2, (t.length + plat) // 2
    t.height_field_raw[x1:x2, y1:y2] = 0
    return t


def stepping_stones_terrain(t, stone_size, stone_distance, max_height, platform_size=1.0, depth=-10):
    ss = int(stone_size / t.horizontal_scale)
    sd = int(stone_distance / t.horizontal_scale)
    mh = int(max_height / t.vertical_scale)
    plat = int(platform_size / t.horizontal_scale)
    levels = np.arange(-mh - 1, mh, step=1)
    t.height_field_raw[:, :] = int(depth / t.vertical_scale)
    x = 0
    while x < t.width:
        y = np.random.randint(0, max(ss, 1))
        while y < t.length:
            t.height_field_raw[x:x + ss, y:y + ss] = np.random.choice(levels)
            y += ss + sd
        x += ss + sd
    x1, x2 = (t.width - plat) // 2, (t.width + plat) // 2
    y1, y2 = (t.length - plat) // 2, (t.length + plat) // 2
    t.height_field_raw[x1:x2, y1:y2] = 0
    return t


def gap_terrain(t, gap_size, platform_size=1.0):  # terrain.py:166-178
    g = int(gap_size / t.horizontal_scale)
    p = int(platform_size / t.horizontal_scale)
    cx, cy = t.length // 2, t.width // 2
    x1 = (t.length - p) // 2
    x2 = x1 + g
    y1 = (t.width - p) // 2
    y2 = y1 + g
    t.height_field_raw[cx - x2:cx + x2, cy - y2:cy + y2] = -1000
    t.height_field_raw[cx - x1:cx + x1, cy - y1:cy + y1] = 0


def pit_terrain(t, depth, platform_size=1.0):  # terrain.py:180-187
    d = int(depth / t.vertical_scale)
    p = int(platform_size / t.horizontal_scale / 2)
    x1, x2 = t.length // 2 - p, t.length // 2 + p
    y1, y2 = t.width // 2 - p, t.width // 2 + p
    t.height_field_raw[x1:x2, y1:y2] = -d


def trimesh_vertex_moves(height_field_raw, horizontal_scale, vertical_scale, slope_threshold):
    """The slope correction of isaacgym.terrain_utils.convert_heightfield_to_trimesh (called at
    terrain.py:70-73 with cfg.slope_treshold, legged_robot_config.py:68): a vertex whose neighbour
    along x, y or the cell diagonal rises by more than slope_threshold * horizontal_scale moves one
    cell toward it, so a steep one-cell ramp becomes a vertical wall.  Returns the per-vertex move
    (dx, dy) in cells, int8 [rows, cols] each, in {-1, 0, 1} (restated from the published
    algorithm; the library is absent: parity unpinned).  Heights are compared as int32 (the int16
    differences of realistic terrains never wrap)."""
    hf = np.asarray(height_field_raw).astype(np.int32)
    R, Cc = hf.shape
    thr = slope_threshold * (horizontal_scale / vertical_scale)   # (the library's `*=` order)
    move_x = np.zeros((R, Cc), np.int32)
    move_y = np.zeros((R, Cc), np.int32)
    move_c = np.zeros((R, Cc), np.int32)
    move_x[:R - 1, :] += hf[1:, :] - hf[:R - 1, :] > thr
    move_x[1:, :] -= hf[:R - 1, :] - hf[1:, :] > thr
    move_y[:, :Cc - 1] += hf[:, 1:] - hf[:, :Cc - 1] > thr
    move_y[:, 1:] -= hf[:, :Cc - 1] - hf[:, 1:] > thr
    move_c[:R - 1, :Cc - 1] += hf[1:, 1:] - hf[:R - 1, :Cc - 1] > thr
    move_c[1:, 1:] -= hf[:R - 1, :Cc - 1] - hf[1:, 1:] > thr
    dx = move_x + move_c * (move_x == 0)
    dy = move_y + move_c * (move_y == 0)
    return dx.astype(np.int8), dy.astype(np.int8)


def convert_heightfield_to_trimesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    """isaacgym.terrain_utils.convert_heightfield_to_trimesh, vectorised (terrain.py:70-73): vertices
    float32 [rows * cols, 3] (grid x = row * horizontal_scale, y = col * horizontal_scale, as
    np.linspace, + the slope-correction moves; z = height * vertical_scale) and triangles uint32
    [2 (rows - 1)(cols - 1), 3], two per cell: (v00, v11, v01), (v00, v10, v11).  Parity UNPINNED
    (isaacgym absent); tests check the construction's invariants."""
    hf = np.asarray(height_field_raw)
    R, Cc = hf.shape
    y = np.linspace(0, (Cc - 1) * horizontal_scale, Cc)
    x = np.linspace(0, (R - 1) * horizontal_scale, R)
    yy, xx = np.meshgrid(y, x)
    if slope_threshold is not None:
        dx, dy = trimesh_vertex_moves(hf, horizontal_scale, vertical_scale, slope_threshold)
        xx = xx + dx * horizontal_scale
        yy = yy + dy * horizontal_scale
    vertices = np.zeros((R * Cc, 3), dtype=np.float32)
    vertices[:, 0] = xx.flatten()
    vertices[:, 1] = yy.flatten()
    vertices[:, 2] = hf.flatten() * vertical_scale
    i = np.arange(R - 1, dtype=np.int64)[:, None]
    j = np.arange(Cc - 1, dtype=np.int64)[None, :]
    ind0 = (i * Cc + j).ravel()
    ind1, ind2 = ind0 + 1, ind0 + Cc
    ind3 = ind2 + 1
    triangles = np.empty((2 * ind0.size, 3), dtype=np.uint32)
    triangles[0::2] = np.stack([ind0, ind3, ind1], 1)
    triangles[1::2] = np.stack([ind0, ind2, ind3], 1)
    return vertices, triangles


def trimesh_contact_tables(dx, dy):
    """The physics kernels' view of the corrected mesh: per-vertex move code (dx + 1) * 3 + (dy + 1)
    (4 = unmoved) and a per-cell flag = some vertex of the 4 x 4 block around cell (i, j) (rows
    i-1 .. i+2, cols j-1 .. j+2) moved, i.e. a query in that cell may be near a corrected (vertical)
    face and takes the closest-point query over the neighbouring triangles."""
    code = ((dx.astype(np.int16) + 1) * 3 + (dy.astype(np.int16) + 1)).astype(np.int8)
    moved = (dx != 0) | (dy != 0)
    R, Cc = moved.shape
    pad = np.zeros((R + 3, Cc + 3), dtype=bool)
    pad[1:R + 1, 1:Cc + 1] = moved
    flag = np.zeros((R, Cc), dtype=bool)
    for a in range(4):
        for b in range(4):
            flag |= pad[a:a + R, b:b + Cc]
    return code, flag.astype(np.int8)


class Terrain:
    """terrain.py:38-164."""

    def __init__(self, cfg, num_robots):
        self.cfg = cfg
        self.num_robots = num_robots
        self.type = cfg.mesh_type
        if self.type in ("none", "plane"):
            return
        self.env_length = cfg.terrain_length
        self.env_width = cfg.terrain_width
        self.proportions = [np.sum(cfg.terrain_proportions[:i + 1]) for i in range(len(cfg.terrain_proportions))]
        cfg.num_sub_terrains = cfg.num_rows * cfg.num_cols
        self.env_origins = np.zeros((cfg.num_rows, cfg.num_cols, 3))
        self.width_per_env_pixels = int(self.env_width / cfg.horizontal_scale)
        self.length_per_env_pixels = int(self.env_length / cfg.horizontal_scale)
        self.border = int(cfg.border_size / cfg.horizontal_scale)
        self.tot_cols = int(cfg.num_cols * self.width_per_env_pixels) + 2 * self.border
        self.tot_rows = int(cfg.num_rows * self.length_per_env_pixels) + 2 * self.border
        self.height_field_raw = np.zeros((self.tot_rows, self.tot_cols), dtype=np.int16)
        if cfg.curriculum:
            self._curriculum()
        elif cfg.selected:
            self._selected()
        else:
            self._randomized()
        self.heightsamples = self.height_field_raw
        if self.type == "trimesh":   # terrain.py:70-73
            self.vertices, self.triangles = convert_heightfield_to_trimesh(
                self.height_field_raw, cfg.horizontal_scale, cfg.vertical_scale, cfg.slope_treshold)
            if cfg.slope_treshold is not None:
                dx, dy = trimesh_vertex_moves(self.height_field_raw, cfg.horizontal_scale, cfg.vertical_scale,
                                              cfg.slope_treshold)
                self.vertex_moves, self.wall_flags = trimesh_contact_tables(dx, dy)

    def _randomized(self):
        for k in range(self.cfg.num_sub_terrains):
            i, j = np.unravel_index(k, (self.cfg.num_rows, self.cfg.num_cols))
            choice = np.random.uniform(0, 1)
            difficulty = np.random.choice([0.5, 0.75, 0.9])
            self._add(self.make_terrain(choice, difficulty), i, j)

    def _curriculum(self):
        for j in range(self.cfg.num_cols):
            for i in range(self.cfg.num_rows):
                self._add(self.make_terrain(j / self.cfg.num_cols + 0.001, i / self.cfg.num_rows), i, j)

    def _selected(self):
        kwargs = dict(self.cfg.terrain_kwargs)
        fn = {"pyramid_sloped_terrain": pyramid_sloped_terrain, "random_uniform_terrain": random_uniform_terrain,
              "pyramid_stairs_terrain": pyramid_stairs_terrain,
              "discrete_obstacles_terrain": discrete_obstacles_terrain,
              "stepping_stones_terrain": stepping_stones_terrain}[kwargs.pop("type").split(".")[-1]]
        for k in range(self.cfg.num_sub_terrains):
            i, j = np.unravel_index(k, (self.cfg.num_rows, self.cfg.num_cols))
            t = SubTerrain(self.width_per_env_pixels, self.width_per_env_pixels, self.cfg.vertical_scale,
                           self.cfg.horizontal_scale)
            fn(t, **kwargs.get("terrain_kwargs", kwargs))
            self._add(t, i, j)

    def make_terrain(self, choice, difficulty):  # terrain.py:109-145
        t = SubTerrain(self.width_per_env_pixels, self.width_per_env_pixels, self.cfg.vertical_scale,
                       self.cfg.horizontal_scale)
        slope = difficulty * 0.4
        step_height = 0.05 + 0.18 * difficulty
        obst_height = 0.05 + difficulty * 0.2
        stone_size = 1.5 * (1.05 - difficulty)
        stone_distance = 0.05 if difficulty == 0 else 0.1
        p = self.proportions + [1.0] * (7 - len(self.proportions))
        if choice < p[0]:
            if choice < p[0] / 2:
                slope *= -1
            pyramid_sloped_terrain(t, slope=slope, platform_size=3.)
        elif choice < p[1]:
            pyramid_sloped_terrain(t, slope=slope, platform_size=3.)
            random_uniform_terrain(t, min_height=-0.05, max_height=0.05, step=0.005, downsampled_scale=0.2)
        elif choice < p[3]:
            if choice < p[2]:
                step_height *= -1
            pyramid_stairs_terrain(t, step_width=0.31, step_height=step_height, platform_size=3.)
        elif choice < p[4]:
            discrete_obstacles_terrain(t, obst_height, 1., 2., 20, platform_size=3.)
        elif choice < p[5]:
            stepping_stones_terrain(t, stone_size=stone_size, stone_distance=stone_distance, max_height=0.,
                                    platform_size=4.)
        elif choice < p[6]:
            gap_terrain(t, gap_size=1. * difficulty, platform_size=3.)
        else:
            pit_terrain(t, depth=1. * difficulty, platform_size=4.)
        return t

    def _add(self, t, row, col):  # terrain.py:147-164
        sx = self.border + row * self.length_per_env_pixels
        sy = self.border + col * self.width_per_env_pixels
        self.height_field_raw[sx:sx + self.length_per_env_pixels, sy:sy + self.width_per_env_pixels] = t.height_field_raw
        ox, oy = (row + 0.5) * self.env_length, (col + 0.5) * self.env_width
        x1 = int((self.env_length / 2. - 1) / t.horizontal_scale)
        x2 = int((self.env_length / 2. + 1) / t.horizontal_scale)
        y1 = int((self.env_width / 2. - 1) / t.horizontal_scale)
        y2 = int((self.env_width / 2. + 1) / t.horizontal_scale)
        oz = np.max(t.height_field_raw[x1:x2, y1:y2]) * t.vertical_scale
        self.env_origins[row, col] = [ox, oy, oz]
