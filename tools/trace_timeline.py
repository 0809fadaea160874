"""Sweep timeline from a rocprofv3 kernel trace (CPU; reads the CSV only).

    python tools/trace_timeline.py run_kernel_trace.csv [--last N]

For each of the last N sweep launches: its duration, the idle gap before it
(previous sweep's end to its start), and the ELBO kernels (cov / pairs /
nodes) of the same window -- when they started, when they ended relative to
the sweep's end, and how long they ran.  A sweep whose workgroups leave no
room on the CUs (kind 22 at config 5: every workgroup holds the main
workgroup's 137 KB of LDS) starves the ELBO kernels queued beside it; they
finish after it, and the host launches the next sweep only after reading
their sums, which is the gap this prints.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 8
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows if "ame_" in r["Kernel_Name"])
    sweeps = [e for e in ev if "sweep" in e[2]]
    if len(sweeps) < 2:
        print("fewer than two sweeps in", path)
        return
    sel = sweeps[-(last + 1):]
    print(f"{'sweep ms':>9} {'gap ms':>7} {'period':>7}  ELBO kernels in the window "
          "(name: start after sweep start / end after sweep end / duration, ms)")
    gaps, periods = [], []
    for prev, cur in zip(sel, sel[1:]):
        gap = (cur[0] - prev[1]) / 1e6
        per = (cur[0] - prev[0]) / 1e6
        win = [e for e in ev if "sweep" not in e[2] and "final" not in e[2] and prev[0] <= e[0] < cur[0]]
        desc = ", ".join(f"{e[2].split('<')[0].split('(')[0].replace('void ', '')}: "
                         f"{(e[0] - prev[0]) / 1e6:.2f}/{(e[1] - prev[1]) / 1e6:+.2f}/{(e[1] - e[0]) / 1e6:.2f}"
                         for e in win)
        print(f"{(prev[1] - prev[0]) / 1e6:9.3f} {gap:7.3f} {per:7.3f}  {desc}")
        gaps.append(gap)
        periods.append(per)
    print(f"mean period {sum(periods) / len(periods):.3f} ms, mean gap {sum(gaps) / len(gaps):.3f} ms "
          f"({100 * sum(gaps) / sum(periods):.1f} % of the period)")


if __name__ == "__main__":
    main()
