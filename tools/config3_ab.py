"""A/B of the configs[3] (Rajagopal 80-muscle, generic interpreter) line
over environment variants read at mh_create, e.g. the excitation lanes
filled by k_exc_lanes (default) against a full DAE evaluation of every lane
(MOCOHIP_EXC_LANES=0), or eval_g's workspace in LDS (MOCOHIP_G_LDS=8).
One JSON line per variant.
    python tools/config3_ab.py [N] ["K=V[,K=V];K=V..." default
        "MOCOHIP_EXC_LANES=1;MOCOHIP_EXC_LANES=0"]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    spec = sys.argv[2] if len(sys.argv) > 2 else "MOCOHIP_EXC_LANES=1;MOCOHIP_EXC_LANES=0"
    variants = [dict(kv.split("=") for kv in v.split(",")) for v in spec.split(";")]
    sys.argv = [sys.argv[0], "--steps", "2000", "--no-cpu-baseline", "--config3", str(N)]
    args = bench.parse()
    cx = bench.Ctx(args)
    for variant in variants:
        os.environ.update(variant)
        line = bench.config3_line(cx, args)
        line["env"] = variant
        for k in variant:
            os.environ.pop(k)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
