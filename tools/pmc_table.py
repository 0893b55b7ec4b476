"""Per-kernel PMC table from rocprofv3 --pmc passes (rocpd sqlite) under one directory.

    python tools/pmc_table.py DIR    # DIR/p<i>_<kernel>/**/*.db, one pass per sub-directory

Prints, per kernel name and counter, the mean value per dispatch (counters summed over the
dispatch's XCDs / SEs as rocprofv3 reports them)."""
import collections
import glob
import os
import re
import sqlite3
import sys


def rows(db):
    """(kernel name, counter, value, dispatch id, duration ns) per counter record."""
    con = sqlite3.connect(db)
    return list(con.execute("select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"))


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(dict))
    dur = collections.defaultdict(dict)
    for db in sorted(glob.glob(os.path.join(d, "p*", "**", "*.db"), recursive=True)):
        for kname, counter, value, ev, ns in rows(db):
            k = re.sub(r"\(.*$", "", kname.replace("(anonymous namespace)::", "").replace("srk::", ""))
            key = (db, ev)
            acc[k][counter][key] = acc[k][counter].get(key, 0.0) + float(value)
            dur[k][key] = float(ns)
    for k, cs in sorted(acc.items()):
        if not any(x in k for x in ("mfcc", "fbank", "spec", "gemm", "gru", "conv", "bn_", "colsum", "pool", "splitk")):
            continue
        ds = list(dur[k].values())
        print("%s   (mean dispatch duration %.1f us)" % (k, sum(ds) / len(ds) / 1e3))
        for c, evs in sorted(cs.items()):
            vals = list(evs.values())
            print("  %-28s %16.1f  (dispatches %d)" % (c, sum(vals) / len(vals), len(vals)))


if __name__ == "__main__":
    main(sys.argv[1])
