"""URDF -> lgx robot model description (container-only data tool).

Reads a legged-robot URDF (the reference's assets, e.g.
/root/reference/resources/robots/go1/urdf/go1.urdf) and writes the compact JSON model
that `legged_gym_amd.sim.model` turns into the C-ABI `lgx_model` struct.  The JSON is
*data* derived from the URDF (masses, inertias, joint frames, limits, collision
primitives); no URDF text is copied into the repo.

Semantics reproduced from the Isaac Gym asset importer as configured by the reference
(`legged_robot.py:658-673`, `legged_robot_config.py:102-122`):
  * collapse_fixed_joints=True: links joined by fixed joints are merged into one rigid
    body (mass, COM and inertia composed), except joints marked dont_collapse="true",
    which keep their child as a separate *reporting* body (the feet).  Dynamically the
    dont_collapse child is rigidly attached, so its inertia is merged into the moving
    parent body here and it only keeps its own index in the contact-force tensor.
  * body / DOF order: depth-first, children visited in name order (Isaac Gym convention,
    FL < FR < RL < RR; evidenced by hip DOF indices [0,3,6,9] at legged_robot.py:966).
  * replace_cylinder_with_capsule=True: cylinders become capsules (segment = cylinder
    length along the cylinder axis, radius unchanged).

Robots with 12 revolute DOFs in serial leg chains hanging off the base: 4 legs x 3 joints (the
quadrupeds) or 2 legs x 6 joints (Cassie); `leg_dof` in the JSON.  The root body keeps its root
link's name ("base" for the quadrupeds, "pelvis" for Cassie), as Isaac Gym names a collapsed body
after its root link (legged_robot.py:678-680 matches termination bodies by substring of these names).

Usage:  python tools/urdf_model.py <urdf> <out.json> <name>
"""
import json
import math
import sys
import xml.etree.ElementTree as ET

import numpy as np


def rpy_to_mat(r, p, y):
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return rz @ ry @ rx


def parse_origin(el):
    if el is None:
        return np.eye(3), np.zeros(3)
    xyz = np.array([float(v) for v in el.get("xyz", "0 0 0").split()])
    rpy = [float(v) for v in el.get("rpy", "0 0 0").split()]
    return rpy_to_mat(*rpy), xyz


class Link:
    def __init__(self, el):
        self.name = el.get("name")
        inert = el.find("inertial")
        self.mass = 0.0
        self.com = np.zeros(3)
        self.inertia = np.zeros((3, 3))
        if inert is not None:
            R, t = parse_origin(inert.find("origin"))
            self.mass = float(inert.find("mass").get("value"))
            i = inert.find("inertia")
            g = lambda k: float(i.get(k, "0"))
            I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")], [g("ixz"), g("iyz"), g("izz")]])
            self.com = t
            self.inertia = R @ I @ R.T
        self.shapes = []  # (kind, R, t, params)
        for c in el.findall("collision"):
            R, t = parse_origin(c.find("origin"))
            geo = c.find("geometry")
            for kind in ("sphere", "box", "cylinder", "capsule", "mesh"):
                g = geo.find(kind)
                if g is not None:
                    self.shapes.append((kind, R, t, dict(g.attrib)))


def compose_inertia(bodies):
    """bodies: list of (mass, com, inertia_about_com) in a common frame."""
    m = sum(b[0] for b in bodies)
    if m <= 0:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    c = sum(b[0] * b[1] for b in bodies) / m
    I = np.zeros((3, 3))
    for mi, ci, Ii in bodies:
        d = ci - c
        I += Ii + mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return m, c, I


def shape_points(kind, R, t, params):
    """Contact primitives of one collision shape: list of (point, radius)."""
    if kind == "sphere":
        return [(t, float(params["radius"]))]
    if kind in ("cylinder", "capsule"):
        L, r = float(params["length"]), float(params["radius"])
        axis = R @ np.array([0.0, 0.0, 1.0])  # URDF cylinder axis = local z
        n = max(2, min(5, int(math.ceil(L / (2 * r))) + 1))  # <=5 spheres per capsule
        return [(t + axis * (-L / 2 + L * k / (n - 1)), r) for k in range(n)]
    if kind == "box":
        sx, sy, sz = [float(v) / 2 for v in params["size"].split()]
        if max(sx, sy, sz) < 0.005:  # sub-5mm placeholder boxes (imu/base stubs)
            return []
        pts = []
        for ix in (-1, 1):
            for iy in (-1, 1):
                for iz in (-1, 1):
                    pts.append((t + R @ np.array([ix * sx, iy * sy, iz * sz]), 0.0))
        return pts
    return []  # meshes are not collision primitives for the lgx contact model


def build(urdf_path, name):
    root = ET.parse(urdf_path).getroot()
    links = {l.get("name"): Link(l) for l in root.findall("link")}
    joints = []
    for j in root.findall("joint"):
        R, t = parse_origin(j.find("origin"))
        ax = j.find("axis")
        axis = np.array([float(v) for v in ax.get("xyz").split()]) if ax is not None else np.array([1.0, 0, 0])
        lim = j.find("limit")
        joints.append(dict(
            name=j.get("name"), type=j.get("type"), parent=j.find("parent").get("link"),
            child=j.find("child").get("link"), R=R, t=t, axis=axis / np.linalg.norm(axis),
            dont_collapse=j.get("dont_collapse", "false") == "true",
            lower=float(lim.get("lower", "0")) if lim is not None else 0.0,
            upper=float(lim.get("upper", "0")) if lim is not None else 0.0,
            effort=float(lim.get("effort", "0")) if lim is not None else 0.0,
            velocity=float(lim.get("velocity", "0")) if lim is not None else 0.0))
    children = {}
    for j in joints:
        children.setdefault(j["parent"], []).append(j)
    child_links = {j["child"] for j in joints}
    root_link = [n for n in links if n not in child_links][0]

    # Rigid groups: each group = a body in Isaac Gym's tensor (frame = group root link).
    # members: (link, R_group_link, t_group_link)
    bodies = []      # dicts: name, members, parent_body, joint (None for root / dont_collapse)
    dofs = []

    def visit(link_name, body_idx, R, t):
        bodies[body_idx]["members"].append((link_name, R, t))
        for j in sorted(children.get(link_name, []), key=lambda jj: jj["child"]):
            Rj, tj = R @ j["R"], t + R @ j["t"]
            if j["type"] == "fixed" and not j["dont_collapse"]:
                visit(j["child"], body_idx, Rj, tj)
            else:
                nb = len(bodies)
                bodies.append(dict(name=j["child"], members=[], parent=body_idx, R_pj=Rj, t_pj=tj,
                                   joint=j if j["type"] != "fixed" else None))
                if j["type"] != "fixed":
                    dofs.append(nb)
                visit(j["child"], nb, np.eye(3), np.zeros(3))

    bodies.append(dict(name=root_link, members=[], parent=-1, R_pj=np.eye(3), t_pj=np.zeros(3), joint=None))
    visit(root_link, 0, np.eye(3), np.zeros(3))
    # Isaac Gym names a collapsed body after its root link (the quadrupeds: "base", Cassie: "pelvis").
    for b in bodies:
        props = []
        pts = []
        for (ln, R, t) in b["members"]:
            L = links[ln]
            if L.mass > 0:
                props.append((L.mass, t + R @ L.com, R @ L.inertia @ R.T))
            for (kind, Rs, ts, params) in L.shapes:
                for (p, r) in shape_points(kind, R @ Rs, t + R @ ts, params):
                    pts.append((p, r))
        b["mass"], b["com"], b["inertia"] = compose_inertia(props)
        b["points"] = pts

    nb = len(bodies)
    assert len(dofs) == 12, f"expected 12 revolute DOFs, got {len(dofs)}"
    # legs: the children of the base that start a serial chain (4 x 3 DOFs or 2 x 6), in order
    leg_roots = [i for i in dofs if bodies[i]["parent"] == 0]
    assert len(leg_roots) in (2, 4), leg_roots
    leg_dof = 12 // len(leg_roots)
    dyn = [0]            # dyn body 0 = base, then per leg its chain's moving bodies
    report_to_dyn = {0: (0, np.eye(3), np.zeros(3))}
    joint_rows = []
    for leg, b0 in enumerate(leg_roots):
        chain = [b0]
        while len(chain) < leg_dof:
            nxt = [i for i in dofs if bodies[i]["parent"] == chain[-1]]
            assert len(nxt) == 1
            chain.append(nxt[0])
        for k, bi in enumerate(chain):
            dyn.append(bi)
            j = bodies[bi]["joint"]
            joint_rows.append(dict(name=j["name"], R=bodies[bi]["R_pj"], t=bodies[bi]["t_pj"], axis=j["axis"],
                                   lower=j["lower"], upper=j["upper"], effort=j["effort"], velocity=j["velocity"]))
            report_to_dyn[bi] = (1 + leg_dof * leg + k, np.eye(3), np.zeros(3))
    # fixed (dont_collapse) bodies -> rigidly attached to their moving parent
    for bi, b in enumerate(bodies):
        if bi in report_to_dyn:
            continue
        p = b["parent"]
        while p not in report_to_dyn:
            p = bodies[p]["parent"]
        d, Rp, tp = report_to_dyn[p]
        report_to_dyn[bi] = (d, Rp @ b["R_pj"], tp + Rp @ b["t_pj"])
    # merged dynamic inertias (attached reporting bodies folded into their dyn body)
    dyn_props = {d: [] for d in range(13)}
    points = []
    for bi, b in enumerate(bodies):
        d, R, t = report_to_dyn[bi]
        if b["mass"] > 0:
            dyn_props[d].append((b["mass"], t + R @ b["com"], R @ b["inertia"] @ R.T))
        for (p, r) in b["points"]:
            points.append(dict(report_body=bi, dyn_body=d, pos=(t + R @ p).tolist(), radius=r))
    dyn_out = []
    for d in range(13):
        m, c, I = compose_inertia(dyn_props[d])
        dyn_out.append(dict(name=bodies[dyn[d]]["name"], mass=m, com=c.tolist(),
                            inertia=[I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]))
    body_names = [b["name"] for b in bodies]
    out = dict(
        name=name,
        leg_dof=leg_dof,
        body_names=body_names,
        dof_names=[j["name"] for j in joint_rows],
        joints=[dict(name=j["name"], rot=j["R"].reshape(-1).tolist(), pos=j["t"].tolist(), axis=j["axis"].tolist(),
                     lower=j["lower"], upper=j["upper"], effort=j["effort"], velocity=j["velocity"]) for j in joint_rows],
        dyn_bodies=dyn_out,
        report_bodies=[dict(name=body_names[bi], dyn_body=report_to_dyn[bi][0], mass=bodies[bi]["mass"],
                            rot=report_to_dyn[bi][1].reshape(-1).tolist(), pos=report_to_dyn[bi][2].tolist())
                       for bi in range(nb)],
        contact_points=points,
    )
    return out


if __name__ == "__main__":
    urdf, dst, name = sys.argv[1:4]
    m = build(urdf, name)
    with open(dst, "w") as f:
        json.dump(m, f, indent=1)
    print(name, "bodies", m["body_names"])
    print("dofs", m["dof_names"])
    print("total mass", sum(b["mass"] for b in m["dyn_bodies"]), "contact points", len(m["contact_points"]))
