"""Is the headline step host-bound?  For the bench's separate-mode step
(gait10dof18musc MocoTrack N=200, device pointers, async calls) print:
  * enqueue_us: host time per step to enqueue K steps (no synchronize inside);
  * wall_us:    wall time per step including the final synchronize;
  * the Python + ctypes cost of one entry call that launches nothing
    (mh_set_async).
If enqueue_us ~= wall_us the GPU waits for the host."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))

import bench  # noqa: E402


def main():
    import torch
    args = bench.parse()
    cx = bench.Ctx(args)
    from mocohip import configs
    st = configs.gait10dof18musc(200, fd_scheme=args.fd)
    nlp = bench.make_nlp(cx, st)
    x = bench.track_iterate(nlp, 0)
    sep, fused, keep = bench.device_steps(cx, nlp, x)
    for name, step in (("separate", sep), ("fused", fused)):
        for _ in range(2000):
            step()
        torch.cuda.synchronize()
        for k in (200, 2000, 10000):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"{name:9s} k={k:6d} enqueue_us {1e6 * (t1 - t0) / k:7.2f} wall_us {1e6 * (t2 - t0) / k:7.2f}",
                  flush=True)
    # the Python + ctypes cost of one entry call alone
    import ctypes as C
    t0 = time.perf_counter()
    for _ in range(100000):
        nlp._check(nlp.lib.mh_set_async(nlp.ctx, C.c_int(1)))
    print(f"ctypes entry call (mh_set_async) us {1e6 * (time.perf_counter() - t0) / 100000:.3f}")


if __name__ == "__main__":
    main()
