"""Diagnostic: time the HostGather device-to-host copy alone (pinned shared
buffer, hipMemcpyAsync on the torch stream) for a given number of doubles."""
import sys
import time

import torch

sys.path.insert(0, "opensim-moco_amd")
from mocohip.distributed import HostGather  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 41146036
dev = torch.device("cuda", 0)
v = torch.arange(n, dtype=torch.float64, device=dev)
g = torch.zeros(1, dtype=torch.float64, device=dev)
hg = HostGather("d2hcheck", 1, n, (0, 1), (0, n), 0, lambda: None, pin=True)
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    hg.copy_from_device_async(g.data_ptr(), v.data_ptr(), s)
torch.cuda.synchronize()
t0 = time.perf_counter()
K = 20
for _ in range(K):
    hg.copy_from_device_async(g.data_ptr(), v.data_ptr(), s)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / K
ok = bool((hg.full_values()[:5] == [0, 1, 2, 3, 4]).all() and hg.full_values()[-1] == n - 1)
print(f"{n} doubles ({8 * n / 1e6:.1f} MB): {el * 1e3:.3f} ms per copy, {8 * n / el / 1e9:.1f} GB/s, content ok {ok}")
hg.close(unlink=True)
