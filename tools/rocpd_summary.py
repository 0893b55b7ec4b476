"""Summarise rocprofv3 result databases (rocpd sqlite) into the text tables committed under profiles/.

    python tools/rocpd_summary.py STATS_DIR [--fetch FETCH_DIR] [--write WRITE_DIR] > profiles/rNN_x.txt

STATS_DIR holds a `--kernel-trace --stats` run; FETCH_DIR / WRITE_DIR hold separate `--pmc FETCH_SIZE` /
`--pmc WRITE_SIZE` passes of the same command (gpurun refuses combined passes; TCC slots do not fit
both anyway).  HBM bytes follow MI355X_MICROARCH.md's gfx950 corrections: FETCH_SIZE (KiB) is doubled
(it tallies wide 128-B streaming reads at 64 B), WRITE_SIZE is taken as reported.
"""
import argparse
import glob
import os
import re
import sqlite3


def _db(d):
    hits = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
    if not hits:
        raise SystemExit("no rocpd database under %s" % d)
    return sqlite3.connect(hits[0])


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(srk::[^)]*\)(, int)?\)?$", "", name)
    return name.replace("srk::", "")[:90]


def kernel_stats(d):
    c = _db(d)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return rows, tot


def pmc(d, counter):
    c = _db(d)
    rows = c.execute("select kernel_name, count(*), avg(value), sum(value) from counters_collection "
                     "where counter_name = ? group by kernel_name", (counter,)).fetchall()
    return {r[0]: (r[1], r[2], r[3]) for r in rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows, tot = kernel_stats(a.stats)
    print("# rocprofv3 --kernel-trace --stats summary (durations in us)")
    print("%-90s %7s %12s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"))
    for name, n, s, av, mn, mx in rows[:a.top]:
        print("%-90s %7d %12.1f %10.2f %10.2f %10.2f %6.2f" % (short(name), n, s / 1e3, av / 1e3, mn / 1e3, mx / 1e3,
                                                                100.0 * s / tot))
    if a.fetch or a.write:
        f = pmc(a.fetch, "FETCH_SIZE") if a.fetch else {}
        w = pmc(a.write, "WRITE_SIZE") if a.write else {}
        print()
        print("# HBM traffic per launch (PMC; FETCH_SIZE x2 per the gfx950 correction, WRITE_SIZE as is), bytes")
        print("%-90s %7s %16s %16s %16s" % ("kernel", "calls", "fetch_B/launch", "write_B/launch", "total_B/launch"))
        names = sorted(set(f) | set(w), key=lambda k: -((f.get(k, (0, 0, 0))[2]) + (w.get(k, (0, 0, 0))[2])))
        for k in names[:a.top]:
            fb = 2.0 * 1024 * f[k][1] if k in f else float("nan")
            wb = 1024 * w[k][1] if k in w else float("nan")
            n = (f.get(k) or w.get(k))[0]
            print("%-90s %7d %16.0f %16.0f %16.0f" % (short(k), n, fb, wb, fb + wb))


if __name__ == "__main__":
    main()
