"""Per-step kernel costs of a decode step: the difference of two rocprofv3 kernel-stats
files of tools/profile_step.py runs with different replay counts (setup cancels out).

    python tools/step_diff.py a_stats.csv b_stats.csv <replays_a> <replays_b> [top]
"""
import csv
import sys


def load(path):
    out = {}
    with open(path) as f:
        rows = list(csv.reader(f))
    for r in rows[1:]:
        name = ",".join(r[:-7])
        out[name] = (int(r[-7]), float(r[-6]))
    return out


def main(a, b, na, nb, top=25):
    A, B = load(a), load(b)
    n = int(nb) - int(na)
    items = []
    for k in set(A) | set(B):
        ca, ta = A.get(k, (0, 0.0))
        cb, tb = B.get(k, (0, 0.0))
        if cb - ca > 0:
            items.append(((tb - ta) / n / 1e3, (cb - ca) / n, k))
    items.sort(reverse=True)
    tot = sum(t for t, _, _ in items)
    print(f"per step: {tot:.1f} us of kernel time over {n} extra replays")
    for t, c, k in items[:int(top)]:
        print(f"{t:9.1f} us {c:7.1f} calls {t / max(c, 1e-9):8.1f} us/call  {k[:100]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
