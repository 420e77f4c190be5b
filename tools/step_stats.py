"""Per-kernel durations of a rocprofv3 kernel-trace directory tree, split by
workgroup size, plus the step's span: for each stop<n> subdirectory of the
argument, the mean duration of each (kernel, workgroup size) over the last
half of the trace (the timed steps), and the mean time from one k_groups
launch of the eval_g stage to the next (one separate-mode step)."""
import collections
import csv
import glob
import os
import sys


def summarize(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[len(rows) // 2:]
    acc = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        acc[(name, r["Workgroup_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = []
    for (name, wg), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        out.append(f"  {name:48s} wg {wg:>5s} calls {len(v):5d} avg {sum(v) / len(v):8.2f} us")
    # step span: consecutive starts of the first kernel of each step (the
    # eval_g stage's k_groups: the k_groups launch that follows a 1024-thread
    # interval kernel)
    starts = []
    prev_wg = None
    for r in rows:
        nm = r["Kernel_Name"]
        if "k_groups" in nm and prev_wg == "1024":
            starts.append(int(r["Start_Timestamp"]))
        if "k_interval" in nm:
            prev_wg = r["Workgroup_Size_X"]
    if len(starts) > 2:
        span = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
        span.sort()
        out.append(f"  step span median {span[len(span) // 2]:.2f} us over {len(span)} steps")
    return out


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "stop*"))):
        print(os.path.basename(d))
        for line in summarize(d):
            print(line)


if __name__ == "__main__":
    main(sys.argv[1])
