"""Scenes of the frozen oracle framebuffers (tests/golden/frames/, make_frame_golden.py).

Geometry is stored in frames/<name>.npz (float32 positions, int32 indices) so the inputs do not
depend on numpy's transcendental functions on the machine that runs the test; everything else
(materials, lights, cameras) is written out here.
"""
import os

import numpy as np

import myraytracer_amd as M
from myraytracer_amd import scenes

HERE = os.path.dirname(os.path.abspath(__file__))
FRAMES = os.path.join(HERE, "frames")
NAMES = ("c1", "mesh5k", "mirror_glass_area")


def geometry(name):
    """Generate (positions float32, indices int32) - used once by make_frame_golden.py."""
    if name == "mesh5k":
        V, F = scenes.icosphere(4)                                    # 5120 tris
        V = V * 1.1 + np.array([0.0, 0.2, 0.0])
        ground = (np.array([[-5.0, -1.0, -5.0], [5.0, -1.0, -5.0], [5.0, -1.0, 5.0], [-5.0, -1.0, 5.0]]),
                  np.array([[0, 2, 1], [0, 3, 2]]))
        P, I = scenes._merge([(V, F), ground])
    elif name == "mirror_glass_area":
        V, F = scenes.icosphere(3)                                    # 1280 tris
        P, I = V * 0.9 + np.array([-1.0, 0.0, -0.5]), F
    else:
        raise KeyError(name)
    return P.astype(np.float32), I.astype(np.int32)


def load_geometry(name):
    d = np.load(os.path.join(FRAMES, f"{name}.npz"), allow_pickle=False)
    return d["positions"].astype(np.float64), d["indices"]


def scene(name):
    if name == "c1":
        return scenes.scene_c1(256, 256)
    P, I = load_geometry(name)
    mesh = M.Mesh(id=1, material="1", positions=P, indices=I, indices_one_based=False, shading_mode="smooth")
    lam = M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.7, 0.55, 0.4), specular=(0.4, 0.4, 0.4), phong=24.0)
    if name == "mesh5k":
        cam = M.Camera(position=(0.0, 1.0, 5.0), gaze_point=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0), fovy=45.0,
                       near_distance=1.0, image_resolution=(200, 150), type="lookAt")
        return M.Scene(cameras=[cam], materials=[lam], objects=[mesh],
                       point_lights=[M.PointLight((4.0, 6.0, 5.0), (30000.0, 30000.0, 30000.0)),
                                     M.PointLight((-5.0, 3.0, 2.0), (8000.0, 9000.0, 12000.0))],
                       ambient_light=(20.0, 20.0, 20.0), background_color=(12.0, 18.0, 30.0),
                       max_recursion_depth=4)
    # mirror mesh, glass sphere, lambertian ground; a point light and two area lights; 4 spp
    mesh.material = "2"
    ground_mat = M.Material(ambient=(0.1, 0.1, 0.1), diffuse=(0.5, 0.6, 0.45), specular=(0.2, 0.2, 0.2), phong=8.0)
    mirror = M.Material(ambient=(0.05, 0.05, 0.05), diffuse=(0.2, 0.2, 0.2), specular=(0.6, 0.6, 0.6), phong=64.0,
                        mirror=(0.75, 0.75, 0.8), type="mirror")
    glass = M.Material(ambient=(0.0, 0.0, 0.0), diffuse=(0.0, 0.0, 0.0), specular=(0.5, 0.5, 0.5), phong=80.0,
                       mirror=(1.0, 1.0, 1.0), ior=1.5, absorption=(0.05, 0.1, 0.2), type="dielectric")
    ground = M.Mesh(id=2, material="1", shading_mode="flat",
                    positions=np.array([[-6.0, -1.0, -6.0], [6.0, -1.0, -6.0], [6.0, -1.0, 6.0], [-6.0, -1.0, 6.0]]),
                    indices=np.array([[1, 3, 2], [1, 4, 3]], np.int32))
    objs = [mesh, ground, M.Sphere(center=(1.3, -0.2, 0.6), radius=0.8, material="3")]
    cam = M.Camera(position=(0.5, 1.6, 5.5), gaze_point=(0.0, -0.2, 0.0), up=(0.0, 1.0, 0.0), fovy=40.0,
                   near_distance=1.0, image_resolution=(96, 72), num_samples=4, type="lookAt")
    return M.Scene(cameras=[cam], materials=[ground_mat, mirror, glass], objects=objs,
                   point_lights=[M.PointLight((3.0, 5.0, 4.0), (20000.0, 20000.0, 20000.0))],
                   area_lights=[M.AreaLight((-2.0, 4.0, 1.0), (0.3, -1.0, 0.0), (400.0, 380.0, 350.0), 1.0),
                                M.AreaLight((2.5, 3.0, -2.0), (-0.5, -1.0, 0.5), (200.0, 220.0, 260.0), 0.6)],
                   ambient_light=(15.0, 15.0, 15.0), background_color=(20.0, 30.0, 45.0), max_recursion_depth=4)

