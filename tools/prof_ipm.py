"""Python profile of the host interior-point code alone (tools/solve_track.py's
problem; the NLP and the device KKT module are built first, then one warm
solve, then the profiled solve): where `seconds_other_host` goes.
    python tools/prof_ipm.py [200|inverse125] [device|host]"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "opensim-moco_amd"))
from mocohip import configs  # noqa: E402
from mocohip.ipm import IpmOptions, solve_ipm  # noqa: E402

what = sys.argv[1] if len(sys.argv) > 1 else "200"
ls = sys.argv[2] if len(sys.argv) > 2 else "device"
st = configs.gait10dof18musc_inverse(int(what[7:] or 125)) if what.startswith("inverse") else \
    configs.gait10dof18musc_track(int(what), muscles=True)
nlp = st.create_nlp()
x0 = st.solver.starting_point(nlp)
o = IpmOptions.from_ipopt(st.solver.ipopt_options())
o.linear_solver = ls
solve_ipm(nlp, x0, o)                      # warm: module build, graphs
pr = cProfile.Profile()
pr.enable()
r = solve_ipm(nlp, x0, o)
pr.disable()
print("wall", round(r.duration, 3), "timings", {k: round(v, 3) if isinstance(v, float) else v for k, v in r.timings.items()})
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
    print(s.getvalue())
