"""A/B of the configs[3] (Rajagopal 80-muscle, generic interpreter) line:
the excitation lanes filled by k_exc_lanes (default) against a full DAE
evaluation of every lane (MOCOHIP_EXC_LANES=0).  One JSON line per variant.
    python tools/config3_ab.py [N]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    sys.argv = [sys.argv[0], "--steps", "2000", "--no-cpu-baseline", "--config3", str(N)]
    args = bench.parse()
    cx = bench.Ctx(args)
    for variant in ("1", "0"):
        os.environ["MOCOHIP_EXC_LANES"] = variant
        line = bench.config3_line(cx, args)
        line["MOCOHIP_EXC_LANES"] = variant
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
