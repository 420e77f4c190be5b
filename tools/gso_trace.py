"""The GSO fiber-velocity residual of rect_fem_r / vasti_r, traced per time
(tests/test_oracle.py::test_muscle_geometry_matches_reference_gso_fiber_
lengths allows 5e-5 there against the reference's 1e-5): per golden time the
normalized fiber length and velocity errors of every right-leg muscle against
std_testGait10dof18musc_GSO_solution_norm_fiber_{length,velocity}.sto, the
preprocessed knee angle, and which knot interval of the MovingPathPoints'
SimmSplines it lies in.  CPU only (the oracle).

    python tools/gso_trace.py > profiles/r05_gso/gso_velocity_trace.txt"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_oracle as T  # noqa: E402  (the GSO restatement the test uses)
from mocohip import configs  # noqa: E402


def main():
    m = configs.gait10dof18musc_model()
    nfl, nfv, te = T._gso_errors(m)
    z = np.load(os.path.join(ROOT, "tests", "golden", "gso_norm_fiber_length.npz"))
    labels = [l.split("/")[-1] for l in z["nfl_labels"][1:]]
    kl, kin = list(z["kin_labels"]), z["kin"]
    t = kin[:, 0]
    sel = (t >= 0.58 - 0.05) & (t <= 1.8 + 0.05)
    t = t[sel]
    p = len(t) // 2
    q = T._gso_lowpass(t[1] - t[0], 6.0, T._gso_pad(np.deg2rad(kin[sel, kl.index("knee_angle_r")]), p))
    tp = T._gso_pad(t, p)
    vi = [mu.name for mu in m.muscles].index("vasti_r")
    knots = next(pt.fx.x for pt in m.muscles[vi].points if pt.fx is not None)
    print("# per muscle: max |normalized fiber length error|, max |normalized fiber velocity error| (time)")
    for c, l in enumerate(labels):
        i = int(np.argmax(nfv[:, c]))
        print(f"# {l:14s} nfl {nfl[:, c].max():.2e}  nfv {nfv[i, c]:.2e} (t = {te[i]:.3f})")
    print(f"# MovingPathPoint SimmSpline knots (knee_angle_r, rad): {knots}")
    print("# time   knee_angle_r(filtered, interp)  knot interval   rect_fem_r nfl / nfv err   vasti_r nfl / nfv err")
    cr, cv = labels.index("rect_fem_r"), labels.index("vasti_r")
    for i, ti in enumerate(te):
        if ti < 1.70:
            continue
        qi = float(np.interp(ti, tp, q))
        k = int(np.searchsorted(knots, qi, side="right")) - 1
        print(f"{ti:.3f}  {qi:+.6e}  [{knots[k]:+.8f}, {knots[k + 1]:+.8f})  "
              f"{nfl[i, cr]:.2e} / {nfv[i, cr]:.2e}   {nfl[i, cv]:.2e} / {nfv[i, cv]:.2e}")


if __name__ == "__main__":
    main()
