#!/usr/bin/env python3
"""Write the engine's scene as MJCF (include/factorysim.h fm_scene_mjcf) for a MuJoCo cross-check.

usage: python tools/export_mjcf.py --arms 2 --objects 4 --seed 42 [--meshdir DIR] -o scene.xml
then, where MuJoCo is installed:  mujoco.MjModel.from_xml_path("scene.xml")
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from factory_marl_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--arms", type=int, default=2)
ap.add_argument("--objects", type=int, default=10)
ap.add_argument("--seed", type=int, default=42)
ap.add_argument("--meshdir", default=None, help="directory holding the iiwa14 .obj meshes (optional)")
ap.add_argument("-o", "--out", default="-")
a = ap.parse_args()
xml = _lib.scene_mjcf(a.arms, a.objects, a.seed, a.meshdir)
if a.out == "-":
    sys.stdout.write(xml)
else:
    with open(a.out, "w") as f:
        f.write(xml)
