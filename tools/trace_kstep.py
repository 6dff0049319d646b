"""k_step statistics from a rocprofv3 kernel trace of bench.py, split by phase.

    python tools/trace_kstep.py TRACE.csv --warmup W --steps K --horizon T [--out summary.json] [--rows rows.csv]

TRACE.csv may also be a --rows file written by an earlier run (profiles/ keeps those, so a committed summary
can be recomputed from the tree).

bench.py runs W warm-up iterations, then K timed ones, each with T env-step
launches, plus (for graph rollouts) one instrumented rollout afterwards.  The
trace's k_step launches are therefore, in order: W*T warm-up, K*T timed, the
rest after.  For every group the summary gives count / mean / median / stdev /
min / max of the kernel durations, and how many launches overlap a k_pregen
dispatch on the side stream (the first reset of all mazes queues the
pre-generation of every maze's next maze, ~46 ms at 65,536 mazes, which runs
beside the first rollout).
"""
import argparse
import csv
import json
import statistics as st


def load(path):
    """(kernel, start, end) rows of a rocprofv3 kernel trace, or of a trimmed --rows file (which keeps the
    k_step and k_pregen rows only: the summary recomputes from it unchanged)."""
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def write_rows(path, ks):
    """The trimmed trace: only the k_step and k_pregen dispatches, in start order."""
    keep = sorted([k for k in ks if "k_step" in k[0] or "k_pregen" in k[0]], key=lambda k: k[1])
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Duration_ns"])
        for n, b, e in keep:
            w.writerow([n, b, e, e - b])


def stats(durs_ns):
    if not durs_ns:
        return None
    us = [d / 1e3 for d in durs_ns]
    return dict(count=len(us), mean_us=st.mean(us), median_us=st.median(us),
                stdev_us=st.pstdev(us), min_us=min(us), max_us=max(us))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--horizon", type=int, default=16)
    ap.add_argument("--mazes", type=int, default=65536)
    ap.add_argument("--alg-bytes", type=int, default=1064)
    ap.add_argument("--out")
    ap.add_argument("--rows", help="also write the k_step / k_pregen rows of the trace (a CSV this script reads back)")
    a = ap.parse_args()
    ks = load(a.trace)
    if a.rows:
        write_rows(a.rows, ks)
    step = sorted([k for k in ks if "k_step" in k[0]], key=lambda k: k[1])
    pregen = [(s, e) for n, s, e in ks if "k_pregen" in n]

    def overlaps(s, e):
        return any(ps < e and s < pe for ps, pe in pregen)

    nw, nt = a.warmup * a.horizon, a.steps * a.horizon
    groups = dict(all=step, warmup=step[:nw], timed=step[nw:nw + nt], after=step[nw + nt:])
    res = dict(trace=a.trace, kernel=step[0][0] if step else None, warmup_iters=a.warmup, timed_iters=a.steps,
               horizon=a.horizon, k_pregen_dispatches=len(pregen))
    for g, L in groups.items():
        s = stats([e - b for _, b, e in L])
        if s is None:
            continue
        s["overlapping_k_pregen"] = sum(overlaps(b, e) for _, b, e in L)
        clean = [e - b for _, b, e in L if not overlaps(b, e)]
        s["mean_us_without_pregen_overlap"] = st.mean(clean) / 1e3 if clean else None
        s["frac_of_8TBps_at_mean"] = a.mazes * a.alg_bytes / (s["mean_us"] * 1e-6) / 8e12
        s["frac_of_8TBps_at_median"] = a.mazes * a.alg_bytes / (s["median_us"] * 1e-6) / 8e12
        res[g] = s
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
