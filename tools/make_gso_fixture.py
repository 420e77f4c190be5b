#!/usr/bin/env python
"""Freeze the reference's GSO muscle-geometry golden data as a test fixture
(run once in the container that has /root/reference; the fixture is data:
inputs and expected outputs, no reference source).

  Moco/Archive/Tests/testGait10dof18musc_kinematics.mot
      gait10dof18musc joint kinematics (degrees for rotations), the input of
  Moco/Archive/Tests/std_testGait10dof18musc_GSO_solution_norm_fiber_length.sto
  Moco/Archive/Tests/std_testGait10dof18musc_GSO_solution_norm_fiber_velocity.sto
      and velocities (testGait10dof18musc.cpp:78-98, also at 1e-5): the
      rigid-tendon normalized fiber lengths GlobalStaticOptimization
      computed from them (testGait10dof18musc.cpp:58-77 compares at 1e-5):
      kinematics within [0.58-0.05, 1.8+0.05] s, lowpass 6 Hz
      (testGait10dof18musc_GSO_setup.xml), muscle-tendon lengths of the model,
      GCV-splined and evaluated at the solution times, then
      l~M = sqrt((lMT - lTs)^2 + (lopt sin(alpha_opt))^2) / lopt
      (DeGrooteFregly2016MuscleStandalone.h:207-231).

Output: tests/golden/gso_norm_fiber_length.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "opensim-moco_amd"))
from mocohip.osim import read_storage  # noqa: E402

REF = "/root/reference/Moco/Archive/Tests/"


def main():
    kl, kd, _ = read_storage(REF + "testGait10dof18musc_kinematics.mot")
    gl, gd, _ = read_storage(REF + "std_testGait10dof18musc_GSO_solution_norm_fiber_length.sto")
    vl, vd, _ = read_storage(REF + "std_testGait10dof18musc_GSO_solution_norm_fiber_velocity.sto")
    assert vl == gl and np.array_equal(vd[:, 0], gd[:, 0])
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "gso_norm_fiber_length.npz"),
                        kin_labels=np.array(kl), kin=kd, nfl_labels=np.array(gl), nfl=gd, nfv=vd)


if __name__ == "__main__":
    main()
