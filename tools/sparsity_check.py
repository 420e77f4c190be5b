"""Device vs oracle callback-sparsity detection on a config (diagnostic)."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "opensim-moco_amd"))
from mocohip import configs  # noqa: E402
from mocohip.solver import HipNLP, OracleNLP  # noqa: E402

st = configs.gait10dof18musc(8)
st.solver.optim_sparsity_detection = "random"
rep = st.problem.create_rep()
g1 = HipNLP(rep, st.solver.options())
g2 = HipNLP(rep, st.solver.options())
ref = OracleNLP(rep, st.solver.options())
a, a2, b = g1.callback_sparsity(), g2.callback_sparsity(), ref.callback_sparsity()
W = 1 + g1.NS + g1.NC + g1.NDV
print("nnz gpu", g1.nnz, g2.nnz, "oracle", ref.nnz)
print("pattern sums", a.sum(), a2.sum(), b.sum(), "gpu repeat equal", np.array_equal(a, a2))
d = np.argwhere((a != b).reshape(-1, W))
print("differing pairs", len(d), d[:20].tolist())
