"""Pack the reference's dataset constants into posecnn_amd/data/models.npz.

Data only (no reference code): YCB/LOV 3-D box extents (data/LOV/extents.txt),
the first P=2620 model points of every class (data/LOV/models/*/points.xyz, the
truncation lib/datasets/lov.py:141-158 applies), the LOV symmetry vector
(lib/datasets/lov.py:38), the YCB intrinsics (my_tools/model2.py:226 /
data/LOV/camera.json) and the LINEMOD extents + symmetry
(data/LINEMOD/extents.txt, lib/datasets/linemod.py:44).

Run once in the build container (where /root/reference exists); the .npz is
committed so the GPU box never reads the reference.
"""
import os
import numpy as np

REF = "/root/reference"
LOV_CLASSES = ('__background__', '002_master_chef_can', '003_cracker_box', '004_sugar_box',
               '005_tomato_soup_can', '006_mustard_bottle', '007_tuna_fish_can', '008_pudding_box',
               '009_gelatin_box', '010_potted_meat_can', '011_banana', '019_pitcher_base',
               '021_bleach_cleanser', '024_bowl', '025_mug', '035_power_drill', '036_wood_block',
               '037_scissors', '040_large_marker', '051_large_clamp', '052_extra_large_clamp',
               '061_foam_brick')


def main():
    ext = np.zeros((22, 3), np.float32)
    ext[1:] = np.loadtxt(os.path.join(REF, "data/LOV/extents.txt"))
    pts = [np.loadtxt(os.path.join(REF, "data/LOV/models", c, "points.xyz")) for c in LOV_CLASSES[1:]]
    P = min(p.shape[0] for p in pts)
    points = np.zeros((22, P, 3), np.float32)
    for i, p in enumerate(pts):
        points[i + 1] = p[:P]
    sym = np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1], np.float32)
    K = np.array([[1066.778, 0, 312.9869], [0, 1067.487, 241.3109], [0, 0, 1]], np.float32)
    lm_ext = np.zeros((16, 3), np.float32)
    lm_ext[1:] = np.loadtxt(os.path.join(REF, "data/LINEMOD/extents.txt"))
    lm_sym = np.array([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0], np.float32)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "models.npz")
    np.savez_compressed(out, lov_extents=ext, lov_points=points, lov_symmetry=sym, K=K,
                        linemod_extents=lm_ext, linemod_symmetry=lm_sym)
    print("wrote", out, "P =", P)


if __name__ == "__main__":
    main()
