"""MJCF exporter (include/factorysim.h fm_scene_mjcf) against the reference's scene.

The fixtures ``tests/golden/scene_mjcf_*.json`` were produced by ``tests/golden/gen_mjcf_golden.py``, which
runs the reference's ``challenge_env/scene.py:build_scene`` over the reference's asset XML under a stub
dm_control (attach semantics, default classes, namescopes) and flattens it the way MuJoCo numbers a
compiled model.  The exporter writes the scene from the tables the HIP kernel runs on; this test parses
the exported document, flattens it the same way and requires the same bodies, geoms, joints, sites,
actuators, excludes and equality -- ids, names, world poses at qpos0 (1e-12), sizes, inertias, contact
parameters, ranges, gains.  Host-only (no GPU).  Not covered: names dm_control would give the two
``bucket`` attachments and the cubes' free joints (duplicate / unnamed scopes), and MuJoCo itself
loading the document (MuJoCo is absent here -- parity unpinned for that step).
"""
import glob
import json
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(glob.glob(os.path.join(GOLD, "scene_mjcf_*.json")))


@pytest.fixture(scope="module")
def lib():
    from factory_marl_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfactorysim.so not built")
    return _lib


def vec(s):
    return [float(x) for x in s.split()]


def quat2mat(q):
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def frame(a):
    p = np.array(vec(a.get("pos", "0 0 0")))
    R = quat2mat(vec(a["quat"])) if "quat" in a else np.eye(3)
    return p, R


def flatten(xml):
    root = ET.fromstring(xml)
    bodies = [{"name": "world", "pos": np.zeros(3), "R": np.eye(3)}]
    geoms, joints, sites = [], [], []

    def contents(node, bid, Pw, Rw):
        for c in node:
            a = c.attrib
            if c.tag == "geom":
                p, R = frame(a)
                size = vec(a.get("size", "0 0 0"))
                geoms.append({"name": a.get("name"), "body": bid, "type": a.get("type", "sphere"),
                              "size": (size + [0.0, 0.0, 0.0])[:3], "pos": Pw + Rw @ p, "R": Rw @ R,
                              "collides": not (a.get("contype") == "0" and a.get("conaffinity") == "0"),
                              "friction": vec(a.get("friction", "1 0.005 0.0001")),
                              "solref": vec(a.get("solref", "0.02 1")),
                              "solimp": (vec(a.get("solimp", "0.9 0.95 0.001 0.5 2")) + [0.5, 2.0])[:5],
                              "priority": int(a.get("priority", 0)),
                              "mass": float(a["mass"]) if "mass" in a else None,
                              "rgba": vec(a["rgba"]) if a.get("name", "").startswith("cube") else None})
            elif c.tag in ("joint", "freejoint"):
                jt = "free" if c.tag == "freejoint" else a.get("type", "hinge")
                joints.append({"name": a.get("name"), "type": jt, "body": bid,
                               "axis": Rw @ np.array(vec(a.get("axis", "0 0 1"))),
                               "range": vec(a["range"]) if "range" in a else None,
                               "damping": float(a.get("damping", 0))})
            elif c.tag == "site":
                p, _ = frame(a)
                sites.append({"name": a["name"], "body": bid, "pos": Pw + Rw @ p})
            elif c.tag == "inertial":
                bodies[bid].update(mass=float(a["mass"]), ipos=vec(a["pos"]), diaginertia=vec(a["diaginertia"]),
                                   iR=frame({"quat": a["quat"]} if "quat" in a else {})[1].reshape(-1))
        for c in node:
            if c.tag == "body":
                p, R = frame(c.attrib)
                nb = len(bodies)
                bodies.append({"name": c.attrib.get("name"), "pos": Pw + Rw @ p, "R": Rw @ R})
                contents(c, nb, Pw + Rw @ p, Rw @ R)

    contents(root.find("worldbody"), 0, np.zeros(3), np.eye(3))
    act = []
    for c in root.find("actuator"):
        a = c.attrib
        act.append({"name": a["name"], "target": a.get("joint") or a.get("tendon"), "kind": c.tag,
                    "ctrlrange": vec(a["ctrlrange"]), "gainprm": vec(a["gainprm"]) if "gainprm" in a else None,
                    "biasprm": vec(a["biasprm"]) if "biasprm" in a else None,
                    "kv": float(a["kv"]) if "kv" in a else None,
                    "forcerange": vec(a["forcerange"]) if "forcerange" in a else None})
    excl = [[c.attrib["body1"], c.attrib["body2"]] for c in root.find("contact")]
    eq = [{k: (vec(v) if k.startswith("sol") else v) for k, v in c.attrib.items()} for c in root.find("equality")]
    return dict(bodies=bodies, geoms=geoms, joints=joints, sites=sites, actuators=act, excludes=excl, equality=eq,
                option=root.find("option").attrib)


def named(n):
    # names the fixture pins (dm_control's names for the duplicate bucket scopes / unnamed free joints are not)
    return n is not None and "bucket" not in n


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(p)[11:-5] for p in CASES])
def test_export_matches_reference_scene(lib, path):
    g = json.load(open(path))
    ours = flatten(lib.scene_mjcf(g["A"], g["K"], g["seed"]))
    tol = 1e-12
    # bodies: count, depth-first order, names, world pose at qpos0, inertials
    assert len(ours["bodies"]) == len(g["bodies"])
    for b, (x, y) in enumerate(zip(ours["bodies"], g["bodies"])):
        if named(y["name"]):
            assert x["name"] == y["name"], b
        np.testing.assert_allclose(x["pos"], y["pos"], atol=tol, err_msg=f"body {b} {y['name']}")
        np.testing.assert_allclose(x["R"].reshape(-1), y["R"], atol=tol, err_msg=f"body {b} {y['name']}")
        for k in ("mass", "ipos", "diaginertia", "iR"):
            if k in y:
                np.testing.assert_allclose(x[k], y[k], rtol=1e-15, atol=1e-15, err_msg=f"body {b} {k}")
    # geoms: MuJoCo ids (body order, XML order within a body), names, type, size, pose, contact parameters
    assert len(ours["geoms"]) == len(g["geoms"])
    for i, (x, y) in enumerate(zip(ours["geoms"], g["geoms"])):
        msg = f"geom {i} {y['name']}"
        if named(y["name"]):
            assert x["name"] == y["name"], msg
        assert x["body"] == y["body"] and x["collides"] == y["collides"], msg
        if not y["collides"]:
            continue  # visual mesh slot (placeholder without the mesh files)
        assert x["type"] == y["type"], msg
        n = 1 if y["type"] == "sphere" else 3
        np.testing.assert_allclose(x["size"][:n], y["size"][:n], rtol=1e-15, err_msg=msg)
        np.testing.assert_allclose(x["pos"], y["pos"], atol=tol, err_msg=msg)
        if y["type"] == "box":
            np.testing.assert_allclose(x["R"].reshape(-1), y["R"], atol=tol, err_msg=msg)
        for k in ("friction", "solref", "solimp"):
            np.testing.assert_allclose(x[k], y[k], rtol=1e-15, err_msg=f"{msg} {k}")
        assert x["priority"] == y["priority"], msg
        if y["mass"] is not None:
            assert x["mass"] == pytest.approx(y["mass"], rel=1e-15), msg
        if y["rgba"] is not None:
            np.testing.assert_allclose(x["rgba"], y["rgba"], rtol=0, atol=0, err_msg=msg)
    # joints: qpos / dof order, names the reference looks up, ranges, axes, damping
    assert [j["type"] for j in ours["joints"]] == [j["type"] for j in g["joints"]]
    for x, y in zip(ours["joints"], g["joints"]):
        assert x["body"] == y["body"]
        if y["type"] != "free":
            assert x["name"] == y["name"]
            np.testing.assert_allclose(x["axis"], y["axis"], atol=tol)
            assert x["damping"] == y["damping"]
        if y["range"] is not None:
            np.testing.assert_allclose(x["range"], y["range"], rtol=1e-15)
    # sites the IK policy and the env read
    gs = {s["name"]: s for s in g["sites"]}
    for s in ours["sites"]:
        if named(s["name"]):
            assert s["name"] in gs, s["name"]
            assert s["body"] == gs[s["name"]]["body"]
            np.testing.assert_allclose(s["pos"], gs[s["name"]]["pos"], atol=tol, err_msg=s["name"])
    assert {s for s in gs if named(s)} == {s["name"] for s in ours["sites"] if named(s["name"])}
    # actuators in ctrl order
    assert len(ours["actuators"]) == len(g["actuators"])
    for x, y in zip(ours["actuators"], g["actuators"]):
        assert (x["name"], x["target"], x["kind"]) == (y["name"], y["target"], y["kind"])
        np.testing.assert_allclose(x["ctrlrange"], y["ctrlrange"], rtol=1e-15)
        for k in ("gainprm", "biasprm", "forcerange"):
            if y[k] is not None:
                np.testing.assert_allclose(x[k], y[k], rtol=0)
        assert x["kv"] == y["kv"]
    assert sorted(map(tuple, ours["excludes"])) == sorted(map(tuple, g["excludes"]))
    assert len(ours["equality"]) == len(g["equality"])
    for x, y in zip(ours["equality"], g["equality"]):
        assert (x["joint1"], x["joint2"]) == (y["joint1"], y["joint2"])
        np.testing.assert_allclose(x["solref"], y["solref"])
        np.testing.assert_allclose(x["solimp"][:3], y["solimp"][:3])
    # the reference's solver settings (scene.xml:2 + MuJoCo defaults the kernel implements)
    assert ours["option"]["integrator"] == "implicitfast" and float(ours["option"]["timestep"]) == 0.001
    assert ours["option"]["cone"] == "pyramidal" and ours["option"]["solver"] == "Newton"


def test_export_sizes_match_the_engine(lib):
    """nq / nv / nu of the exported model are the engine's (fm_nq / fm_nv / fm_nu formulas of fm_scene.cpp)."""
    for A, K in [(2, 4), (2, 8), (4, 16), (6, 3)]:
        f = flatten(lib.scene_mjcf(A, K, 1))
        nq = sum({"free": 7, "hinge": 1, "slide": 1}[j["type"]] for j in f["joints"])
        nv = sum({"free": 6, "hinge": 1, "slide": 1}[j["type"]] for j in f["joints"])
        assert (nq, nv, len(f["actuators"])) == (1 + 7 * K + 9 * A, 1 + 6 * K + 9 * A, 1 + 8 * A)


def test_export_with_meshes_keeps_geom_ids(lib):
    a = flatten(lib.scene_mjcf(2, 4, 42))
    b = flatten(lib.scene_mjcf(2, 4, 42, meshdir="/opt/iiwa_assets"))
    assert [g["name"] for g in a["geoms"]] == [g["name"] for g in b["geoms"]]
    assert sum(g["type"] == "mesh" for g in b["geoms"]) == 2 * 15
    root = ET.fromstring(lib.scene_mjcf(2, 4, 42, meshdir="/opt/iiwa_assets"))
    assert root.find("compiler").attrib["meshdir"] == "/opt/iiwa_assets"
    assert len(root.find("asset").findall("mesh")) == 13


def test_export_rejects_bad_scenes(lib):
    from factory_marl_amd._lib import FactorySimError

    with pytest.raises(FactorySimError):
        lib.scene_mjcf(3, 4, 0)
    with pytest.raises(FactorySimError):
        lib.scene_mjcf(2, 0, 0)
