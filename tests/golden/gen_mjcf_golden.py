"""Golden fixture for the MJCF exporter (include/factorysim.h fm_scene_mjcf).

Runs ONLY in the build container (reads /root/reference, read-only).  It imports the reference's own
``challenge_env/scene.py`` under a stub ``dm_control.mjcf`` that parses the reference's asset files
(``assets/scene.xml``, ``conveyor_belt.xml``, ``kuka_iiwa_14/iiwa14.xml``, ``gripper.xml``) with
ElementTree, resolves their default classes and reproduces dm_control's attach semantics (an attached
model becomes an attachment-frame body ``<model>/`` placed at the site or world origin, element names
carry the namescope prefixes, unnamed geoms are ``<scope>//unnamed_geom_<j>``).  ``build_scene`` then
composes the scene exactly as the reference does (table length, cube draws from default_rng(seed),
bucket and arm placement, the 6-arm layout).  The generator flattens the tree the way MuJoCo's
compiler numbers it (bodies depth-first, geoms / joints by body) and records, at qpos0, every body's
world pose, every geom's type / size / world pose / contact parameters / mass / rgba, every joint's
type / range / world axis, every actuator's target and ranges, the contact excludes and the equality.
scene.py's euler angles are taken in radians (dm_control writes a radian compiler into the models it
compiles).  Output: ``tests/golden/scene_mjcf_<A>x<K>_s<seed>.json`` -- data only.

Usage:  python tests/golden/gen_mjcf_golden.py
"""
import json
import os
import sys
import types
import xml.etree.ElementTree as ET

import numpy as np

REF = "/root/reference"
ASSETS = os.path.join(REF, "challenge_env", "challenge_env", "assets")
OUT = os.path.dirname(os.path.abspath(__file__))
CASES = [(2, 4, 42), (2, 10, 7), (4, 16, 3), (6, 5, 11)]


# ----------------------------------------------------------------------------------------------
# a minimal dm_control.mjcf: elements, default classes, attach / namescopes
# ----------------------------------------------------------------------------------------------
class Elem:
    def __init__(self, tag, attrs, parent, model):
        self.tag = tag
        self.attrs = {k: v for k, v in attrs.items()}
        self.children = []
        self.parent = parent
        self.model = model  # owning Root (namescope)
        self.attached = None  # attachment frame: the attached Root

    def add(self, tag, **attrs):
        e = Elem(tag, attrs, self, self.model)
        self.children.append(e)
        return e

    def set_attributes(self, **kw):
        self.attrs.update(kw)

    def attach(self, root):
        # site.attach(model): a frame body in the site's body at the site's pose (dm_control semantics)
        assert self.tag == "site"
        f = Elem("body", {k: self.attrs[k] for k in ("pos", "quat", "euler") if k in self.attrs}, self.parent,
                 self.model)
        f.attached = root
        root.parent_scope = self.model
        self.parent.children.append(f)
        return f

    def find(self, tag, name):
        for e in walk(self.model.worldbody):
            if e.tag == tag and e.attrs.get("name") == name:
                return e
        raise KeyError(name)


class Root:
    def __init__(self, model=None):
        self.name = model
        self.parent_scope = None
        self.worldbody = Elem("worldbody", {}, None, self)
        self.sections = {k: [] for k in ("actuator", "contact", "equality", "tendon")}
        self.defaults = {}  # class -> {tag: attrs}, inheritance already applied
        self.option = {}

    def attach(self, root):
        f = Elem("body", {}, self.worldbody, self)
        f.attached = root
        root.parent_scope = self
        self.worldbody.children.append(f)
        return f

    def find(self, tag, name):
        return self.worldbody.find(tag, name) if tag != "worldbody" else self.worldbody


def walk(e):
    yield e
    for c in e.children:
        yield from walk(c)
    if e.attached is not None:
        yield from walk(e.attached.worldbody)


def _parse_defaults(node, inherited, out, name="main"):
    mine = {t: dict(a) for t, a in inherited.items()}
    for c in node:
        if c.tag != "default":
            mine.setdefault(c.tag, {}).update(c.attrib)
    out[name] = mine
    for c in node:
        if c.tag == "default":
            _parse_defaults(c, mine, out, c.attrib["class"])


def from_path(path):
    tree = ET.parse(path).getroot()
    root = Root(tree.attrib.get("model"))
    for d in tree.findall("default"):
        _parse_defaults(d, {}, root.defaults)

    def build(xnode, parent, cls):
        for c in xnode:
            ccls = c.attrib.get("class", cls)
            attrs = dict(root.defaults.get(ccls, {}).get(c.tag, {})) if ccls else {}
            attrs.update({k: v for k, v in c.attrib.items() if k not in ("class", "childclass")})
            e = Elem(c.tag, attrs, parent, root)
            parent.children.append(e)
            build(c, e, c.attrib.get("childclass", ccls))

    wb = tree.find("worldbody")
    build(wb, root.worldbody, None)
    for sec in root.sections:
        s = tree.find(sec)
        if s is None:
            continue
        for c in s:
            cls = c.attrib.get("class")
            attrs = dict(root.defaults.get(cls, {}).get(c.tag, {})) if cls else {}
            attrs.update({k: v for k, v in c.attrib.items() if k != "class"})
            attrs["__children"] = [dict(g.attrib) for g in c]
            root.sections[sec].append((c.tag, attrs))
    return root


def install_stubs():
    mjcf = types.ModuleType("dm_control.mjcf")
    mjcf.RootElement = Root
    mjcf.from_path = from_path
    dm = types.ModuleType("dm_control")
    dm.mjcf = mjcf
    mj = types.ModuleType("mujoco")
    mj.viewer = types.ModuleType("mujoco.viewer")
    sys.modules.update({"dm_control": dm, "dm_control.mjcf": mjcf, "mujoco": mj, "mujoco.viewer": mj.viewer})


# ----------------------------------------------------------------------------------------------
# flatten like MuJoCo's compiler
# ----------------------------------------------------------------------------------------------
def vec(s, n=None):
    v = [float(x) for x in (s.split() if isinstance(s, str) else s)]
    return v


def quat2mat(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def local_frame(attrs):
    p = np.array(vec(attrs.get("pos", "0 0 0")))
    if "quat" in attrs:
        R = quat2mat(vec(attrs["quat"]))
    elif "euler" in attrs:  # intrinsic xyz (MuJoCo's default eulerseq), radians
        a, b, c = vec(attrs["euler"])
        Rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
        Ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
        Rz = np.array([[np.cos(c), -np.sin(c), 0], [np.sin(c), np.cos(c), 0], [0, 0, 1]])
        R = Rx @ Ry @ Rz
    else:
        R = np.eye(3)
    return p, R


def prefix(root):
    parts = []
    r = root
    while r is not None and r.parent_scope is not None:
        parts.append(r.name)
        r = r.parent_scope
    return "".join(p + "/" for p in reversed(parts))


def flatten(scene):
    bodies, geoms, joints, sites = [], [], [], []
    unnamed = {}

    def full(e, name):
        return prefix(e.model) + name

    def visit_body(e, parent_id, Pw, Rw, frame_of=None):
        bid = len(bodies)
        if frame_of is not None:
            name = prefix(frame_of)
        else:
            name = full(e, e.attrs["name"]) if "name" in e.attrs else None
        bodies.append({"name": name, "parent": parent_id, "pos": Pw.tolist(), "R": Rw.reshape(-1).tolist()})
        kids = list(e.children) + (list(e.attached.worldbody.children) if e.attached is not None else [])
        for c in kids:
            if c.tag == "geom":
                p, R = local_frame(c.attrs)
                if "name" in c.attrs:
                    gname = full(c, c.attrs["name"])
                else:
                    sc = prefix(c.model)
                    j = unnamed.get(sc, 0)
                    unnamed[sc] = j + 1
                    gname = sc + "/unnamed_geom_" + str(j)
                size = vec(c.attrs.get("size", "0 0 0"))
                geoms.append({
                    "name": gname, "body": bid, "type": c.attrs.get("type", "sphere"),
                    "size": (size + [0.0, 0.0, 0.0])[:3], "pos": (Pw + Rw @ p).tolist(),
                    "R": (Rw @ R).reshape(-1).tolist(),
                    "collides": not (c.attrs.get("contype") == "0" and c.attrs.get("conaffinity") == "0"),
                    "friction": vec(c.attrs.get("friction", "1 0.005 0.0001")),
                    "solref": vec(c.attrs.get("solref", "0.02 1")),
                    "solimp": (vec(c.attrs.get("solimp", "0.9 0.95 0.001 0.5 2")) + [0.5, 2.0])[:5],
                    "priority": int(c.attrs.get("priority", 0)),
                    "mass": float(c.attrs["mass"]) if "mass" in c.attrs else None,
                    "rgba": vec(c.attrs["rgba"]) if ("rgba" in c.attrs and c.model.name.startswith("cube")) else None,
                })
            elif c.tag in ("joint", "freejoint"):
                jt = "free" if c.tag == "freejoint" else c.attrs.get("type", "hinge")
                ax = np.array(vec(c.attrs.get("axis", "0 0 1")))
                rng = vec(c.attrs["range"]) if "range" in c.attrs else None
                joints.append({"name": full(c, c.attrs["name"]) if "name" in c.attrs else None, "type": jt,
                               "body": bid, "axis": (Rw @ ax).tolist(), "range": rng,
                               "damping": float(c.attrs.get("damping", 0))})
            elif c.tag == "site":
                p, R = local_frame(c.attrs)
                sites.append({"name": full(c, c.attrs["name"]), "body": bid, "pos": (Pw + Rw @ p).tolist()})
            elif c.tag == "inertial":
                bodies[bid]["mass"] = float(c.attrs["mass"])
                bodies[bid]["ipos"] = vec(c.attrs["pos"])
                bodies[bid]["diaginertia"] = vec(c.attrs["diaginertia"])
                bodies[bid]["iR"] = local_frame({"quat": c.attrs["quat"]} if "quat" in c.attrs else {})[1].reshape(-1).tolist()
        for c in kids:
            if c.tag == "body":
                p, R = local_frame(c.attrs)
                visit_body(c, bid, Pw + Rw @ p, Rw @ R, frame_of=c.attached)

    bodies.append({"name": "world", "parent": -1, "pos": [0, 0, 0], "R": np.eye(3).reshape(-1).tolist()})
    for c in scene.worldbody.children:
        if c.tag == "geom":
            geoms.append({"name": c.attrs.get("name"), "body": 0, "type": c.attrs.get("type"),
                          "size": vec(c.attrs["size"]), "pos": [0, 0, 0], "R": np.eye(3).reshape(-1).tolist(),
                          "collides": True, "friction": [1, 0.005, 0.0001], "solref": [0.02, 1],
                          "solimp": [0.9, 0.95, 0.001, 0.5, 2], "priority": 0, "mass": None, "rgba": None})
    for c in scene.worldbody.children:
        if c.tag == "body":
            p, R = local_frame(c.attrs)
            visit_body(c, 0, p, R, frame_of=c.attached)

    # sections in attach order (a model's own entries, then those of the models attached inside it)
    order = []

    def models_in(root):
        order.append(root)
        for e in walk_own(root.worldbody):
            if e.attached is not None:
                models_in(e.attached)

    def walk_own(e):
        yield e
        for c in e.children:
            yield from walk_own(c)

    models_in(scene)
    actuators, excludes, equality = [], [], []
    for r in order:
        pre = prefix(r)
        for tag, a in r.sections["actuator"]:
            target = a.get("joint") or a.get("tendon")
            actuators.append({"name": pre + a["name"], "target": pre + target, "kind": tag,
                              "ctrlrange": vec(a["ctrlrange"]) if "ctrlrange" in a else None,
                              "gainprm": vec(a.get("gainprm", "")) or None, "biasprm": vec(a.get("biasprm", "")) or None,
                              "kv": float(a["kv"]) if "kv" in a else None,
                              "forcerange": vec(a["forcerange"]) if "forcerange" in a else None})
        for tag, a in r.sections["contact"]:
            excludes.append([pre + a["body1"], pre + a["body2"]])
        for tag, a in r.sections["equality"]:
            equality.append({"joint1": pre + a["joint1"], "joint2": pre + a["joint2"], "solref": vec(a["solref"]),
                             "solimp": vec(a["solimp"])})
    return dict(bodies=bodies, geoms=geoms, joints=joints, sites=sites, actuators=actuators, excludes=excludes,
                equality=equality)


def main():
    install_stubs()
    sys.path.insert(0, os.path.join(REF, "challenge_env"))
    from challenge_env import scene  # the reference's own scene composition

    scene.DIR = ASSETS
    for A, K, seed in CASES:
        m = scene.build_scene(num_objects=K, randomize_objects=True, seed=seed, num_arms=A)
        flat = flatten(m)
        flat.update(A=A, K=K, seed=seed, note="reference challenge_env/scene.py build_scene under a stub "
                    "dm_control.mjcf over the reference's asset XML (tests/golden/gen_mjcf_golden.py)")
        path = os.path.join(OUT, f"scene_mjcf_{A}x{K}_s{seed}.json")
        with open(path, "w") as f:
            json.dump(flat, f, separators=(",", ":"))
        print(path, len(flat["bodies"]), "bodies", len(flat["geoms"]), "geoms", len(flat["joints"]), "joints",
              len(flat["actuators"]), "actuators")


if __name__ == "__main__":
    main()
