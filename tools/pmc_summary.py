"""Per-launch HBM traffic of the hot kernels from rocprofv3 PMC passes
(tools/profile_gpu.sh: FETCH_SIZE and WRITE_SIZE in separate passes).

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of
coalesced streaming reads on gfx950 -> x2; WRITE_SIZE is exact for
coalesced stores.  Calibrated on our own access pattern: k_combine reads
back exactly the T/H slabs k_groups writes, and 2 x FETCH_SIZE(k_combine)
matches WRITE_SIZE(k_groups) (profiles/*/summary.txt).  Units: rocprofv3
reports both counters in KiB.

usage: python tools/pmc_summary.py <prof dir> <workload tag> <out.json>"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {"k_groups": "k_groups<", "k_combine": "k_combine<", "k_transcribe": "k_transcribe(",
           "k_transcribe_gs": "k_transcribe_gs(", "k_interval": "k_interval<", "k_eval": "k_eval<",
           "k_combine_split": "k_combine_split<"}


def _short(name):
    """The table key of a kernel: k_interval's 256-thread instantiation (the
    eval_g launches of the separate step) as k_interval_256."""
    for short, pat in KERNELS.items():
        if pat in name:
            if short == "k_interval" and ", 256>" in name:
                return "k_interval_256"
            return short
    return None


def means(path, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            short = _short(r["Kernel_Name"])
            if short:
                acc[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(d, workload, out):
    fetch = means(os.path.join(d, "pmc_fetch"), "FETCH_SIZE")
    write = means(os.path.join(d, "pmc_write"), "WRITE_SIZE")
    # the separate step's passes (eval_g's own launches: k_interval_256 and
    # its k_groups, which the fused step does not run)
    fs = means(os.path.join(d, "pmc_fetch_sep"), "FETCH_SIZE")
    ws = means(os.path.join(d, "pmc_write_sep"), "WRITE_SIZE")
    for k in ("k_interval_256",):
        if k in fs:
            fetch[k] = fs[k]
        if k in ws:
            write[k] = ws[k]
    ks = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k), write.get(k)
        ks[k] = {"fetch_size_kib": f, "write_size_kib": w,
                 "hbm_bytes": None if f is None or w is None else 2 * f * 1024 + w * 1024}
    with open(out, "w") as fh:
        json.dump({"workload": workload, "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes)",
                   "kernels": ks}, fh, indent=1)
    print(json.dumps(ks, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
