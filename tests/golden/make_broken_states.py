"""Transcribes the reference's "broken state" regression inputs into
tests/golden/broken_states.json (run from the repo root; the reference is only
read as text: every number below is copied from the cited test body).

  unittests/comprehensive/test_HalfCheetahTrajectory.cpp
    :126 NUMERICAL_INSTABILITY      :157 BROKEN_POINT (LCP cache of 3)
    :189 CAPSULE_INTER_PENETRATION  (:234 POS_VEL_ERRORS is the same state)
    :284 POS_VEL_ERRORS_2
  Each loads data/skel/half_cheetah.skel (this package's half_cheetah_world)
  and checks verifyAnalyticalJacobians / verifyVelGradients /
  verifyPosVelJacobian / verifyIdentityMapping at the state.

  unittests/comprehensive/test_AtlasTrajectory.cpp
    :147 BROKEN_1   :236 BROKEN_2   :335 BROKEN_3
  createWorld (:93) loads data/sdf/atlas/atlas_v3_no_head.sdf, whose dof
  order is SdfParser's (dart/utils/sdf/SdfParser.cpp:843-878: links taken in
  std::map name order, each after its parent), stored below as "sdf_bodies"
  (the body each group of dofs belongs to, root FreeJoint first).  The tests
  map it by body name onto this package's Atlas (the box-collider URDF of the
  bench, whose tree order differs).  The 96-entry LCP caches belong to the
  SDF model's 32 mesh-foot contacts; the box-foot model's contact set is a
  different size, for which BoxedLcpConstraintSolver ignores a cache, so they
  are not transcribed.  createWorld's limits (forces +-50 with an unactuated
  root, positions +-10, velocities +-20) do not bind at these states.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
HC = "unittests/comprehensive/test_HalfCheetahTrajectory.cpp"
AT = "unittests/comprehensive/test_AtlasTrajectory.cpp"

HALF_CHEETAH = [
    ("NUMERICAL_INSTABILITY", f"{HC}:126",
     [-5.15992, -0.210083, 8.27897, -0.00318367, 0.513758, -0.0286844, 0.587853, 0.0282165, 0.486934],
     [-2.22286, -6.07728, 0.890211, 9.22385, 3.00743, 1.34837, 9.61029, -2.97553, 9.96726],
     [0, 0, 3.15531, -8.41413, -6.37498, -5.82503, -7.75906, 9.98554, 7.19786],
     []),
    ("BROKEN_POINT", f"{HC}:157",
     [3.21866, -0.465303, 5.9565, -0.487295, -0.969093, 0.0792724, -0.235988, -0.109183, 0.0769134],
     [4.32527, -4.96436, 12.677, 6.0086, -21.5535, 6.76575, 25.5498, -86.1003, 38.0762],
     [-0.0, -0.0, -0.398301, -2.15491, -6.51447, 23.0772, 7.68141, -30.2488, 9.71529],
     [11.9108, 11.8521, 0]),
    ("CAPSULE_INTER_PENETRATION", f"{HC}:189, :234",
     [-8.71924, -0.0564965, -7.58459, 0.291652, -0.587514, 0.200843, 0.255774, 0.802592, -0.201628],
     [2.85676, 8.95689, -1.45436, -8.77701, -3.59597, -2.06459, -7.10815, 3.59627, -20.2623],
     [0, 0, 0.193621, -9.13741, 9.79953, 5.09491, -1.46957, -8.3705, -9.74503],
     []),
    ("POS_VEL_ERRORS_2", f"{HC}:284",
     [-0.0442559, -0.204541, -0.00676443, -0.0591177, -0.0841678, -0.360202, -0.224704, -0.102217, -0.0377656],
     [-0.119657, -0.571126, -0.0161144, -0.257376, -0.0404545, -0.431694, -0.418564, -0.279473, -0.24886],
     [-0.0, -0.0, -0.257804, -0.352182, -0.114889, -0.0418478, -0.261154, -0.208821, -0.0516623],
     []),
]

# dof-owning bodies in atlas_v3_no_head.sdf's SdfParser order (pelvis = root
# FreeJoint, 6 dofs; every other body one revolute dof)
SDF_BODIES = ["pelvis", "ltorso", "mtorso", "utorso",
              "l_clav", "l_scap", "l_uarm", "l_larm", "l_farm",
              "l_uglut", "l_lglut", "l_uleg", "l_lleg", "l_talus", "l_foot", "l_hand",
              "r_clav", "r_scap", "r_uarm", "r_larm", "r_farm",
              "r_uglut", "r_lglut", "r_uleg", "r_lleg", "r_talus", "r_foot", "r_hand"]

ATLAS_FORCE_12 = [0, 0, 0, 0, 0, 0, -7.44122, -1.70693, -5.2703, -2.6099,
                  -5.7076, 0.985185, -6.3785, 0.372082, -9.87066, 7.78529, 0.081559,
                  3.65908, 1.93437, -4.29761, -6.52332, -4.70401, 2.88616, -0.000431554,
                  -3.0544, -4.1798, 2.00762, 7.96103, -8.62058, -5.69036, 7.01415, 4.63665,
                  3.18185]
ATLAS = [
    ("BROKEN_1", f"{AT}:147",
     [-1.571, -0.00288326, 0.00165361, 0.000259454, -0.0102512,
      1.84494e-05, 0.000848932, 0.00334193, 0.00028172, -0.000263459,
      0.000695572, 0.0150866, -0.00288076, -0.0202479, 0.000544379, 0.000227742,
      0.0050451, -0.00294216, 0.000669709, 0.000114237, 0.0646027, -2.75759e-05,
      -7.91484e-05, -0.0106369, 2.12794e-05, 0.0116945, 0.000591883,
      0.000231497, 0.00423308, -0.00163132, -0.000462828, 3.65345e-05,
      0.0220306],
     [-0.0355665, -0.712732, -0.0197312, 0.0644581, -0.00523274,
      -0.0570926, 0.0472622, 0.825493, 0.0338969, -0.0882721, 0.183699, 0.17503,
      -0.649341, 0.0965665, 0.0195836, 0.0421524, 1.19344, -0.665203, 0.184475,
      -0.00623832, 10.9633, 0.0267205, 0.106822, -4.22165, -0.204534, 5.39066,
      0.0195849, 0.0421863, 1.07122, -0.443072, 0.0845663, -0.00623839, 2.65921],
     ATLAS_FORCE_12),
    ("BROKEN_2", f"{AT}:236",
     [-1.57102, -0.00298104, 0.00176851, 0.00027332, -0.0102446,
      2.25516e-05, 0.000838035, 0.00349415, 0.000302042, -0.000268057,
      0.000681061, 0.0150735, -0.00286418, -0.0202515, 0.000771647, 0.000250073,
      0.00527326, -0.00307521, 0.000825464, -2.66419e-05, 0.0646006,
      -3.23823e-05, -6.50984e-05, -0.0106499, 4.97962e-06, 0.011691,
      0.000771647, 0.000250029, 0.00449108, -0.0019256, 0.00045803,
      -2.65981e-05, 0.0220327],
     [-0.0355415, -0.712449, -0.0197237, 0.0644239, -0.00522888,
      -0.0571042, 0.0472592, 0.825169, 0.0338612, -0.0882515, 0.183756,
      0.175005, -0.649385, 0.0966408, 0.0195587, 0.042304, 1.19296, -0.664948,
      0.184412, -0.00625319, 10.9633, 0.0267056, 0.106785, -4.22162, -0.204477,
      5.3907, 0.0195588, 0.0422993, 1.07078, -0.442892, 0.0845375, -0.0062484,
      2.65919],
     ATLAS_FORCE_12),
    ("BROKEN_3", f"{AT}:335",
     [-1.57098, -0.00244077, 0.00131736, 0.000214826, -0.0101934,
      1.85193e-05, 0.000759851, 0.00276811, 0.000261443, -0.00019732,
      0.000574608, 0.0133507, -0.00239568, -0.0184735, 0.000715009, 0.000210485,
      0.00419423, -0.00245556, 0.000653731, -2.188e-05, 0.0532566, -4.87561e-05,
      -0.000114901, -0.00672978, 8.71723e-05, 0.00632901, 0.000715009,
      0.00021045, 0.00353137, -0.00150703, 0.000368055, -2.18447e-05, 0.0189617],
     [-0.0344442, -0.631138, -0.0567461, 0.058374, -0.00398089,
      -0.0513241, 0.0781846, 0.726033, 0.0405993, -0.0707367, 0.106453, 1.72279,
      -0.468507, -1.77798, 0.0566378, 0.0395876, 1.07904, -0.619651, 0.171733,
      -0.0047619, 11.3439, 0.0163738, 0.0498022, -3.92009, -0.0821927, 5.36199,
      0.0566378, 0.0395791, 0.959703, -0.418562, 0.0899755, -0.0047534, 3.07108],
     [0, 0, 0, 0, 0, 0, -2.87179, -0.392243, 1.37066, -6.96699,
      7.84975, -9.84715, -9.55796, 2.85221, 1.37246, -3.28473, 3.33182, 4.61692,
      -1.53041, -8.09531, -1.30448, 4.58172, -6.8179, -4.38499, -9.95055,
      -2.08851, -8.31803, 3.78765, -5.04101, 8.23899, -9.01072, -0.45285,
      -1.28571]),
]


def main():
    out = {"source": "reference unittests, transcribed by tests/golden/make_broken_states.py",
           "half_cheetah": [{"name": n, "source": s, "pos": p, "vel": v, "force": f, "lcp_cache": c}
                            for n, s, p, v, f, c in HALF_CHEETAH],
           "atlas": {"sdf_bodies": SDF_BODIES,
                     "cases": [{"name": n, "source": s, "pos": p, "vel": v, "force": f}
                               for n, s, p, v, f in ATLAS]}}
    for case in out["atlas"]["cases"]:
        assert len(case["pos"]) == len(case["vel"]) == len(case["force"]) == 33
    with open(os.path.join(HERE, "broken_states.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(len(HALF_CHEETAH), "half-cheetah states,", len(ATLAS), "atlas states")


if __name__ == "__main__":
    main()
