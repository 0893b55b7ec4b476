"""Per-phase K1 (mfcc3_kernel) instruction counts from tools/feat_budget.sh's rocprofv3 databases:
SQ_INSTS_* summed over the dispatch, per clip, for each build, and the phase = the difference of two
consecutive builds (stop0 = sample loads + the per-clip epilogue, stop1 = + window / pass A / transpose,
stop2 = + pass B, stop3 = + untangle, full = + mel / dB)."""
import glob
import os
import sqlite3
import sys

CLIPS = 65536
d = sys.argv[1]
rows = {}
for v in ("stop0", "stop1", "stop2", "stop3", "full"):
    acc, n = {}, set()
    for db in glob.glob(os.path.join(d, v, "**", "*.db"), recursive=True):
        con = sqlite3.connect(db)
        for kname, counter, value, ev in con.execute(
                "select kernel_name, counter_name, value, dispatch_id from counters_collection"):
            if "mfcc3_kernel" not in kname:
                continue
            acc.setdefault(counter, {})
            acc[counter][(db, ev)] = acc[counter].get((db, ev), 0.0) + float(value)
            n.add((db, ev))
    rows[v] = {c: sum(x.values()) / max(len(x), 1) / CLIPS for c, x in acc.items()}
cols = ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES",
        "SQ_BUSY_CYCLES")
print("%-8s " % "build" + " ".join("%16s" % c[3:] for c in cols) + "   (per clip)")
for v, r in rows.items():
    print("%-8s " % v + " ".join("%16.1f" % r.get(c, float("nan")) for c in cols))
names = {"stop0": "loads+epilogue", "stop1": "window+passA", "stop2": "passB", "stop3": "untangle", "full": "mel+dB"}
prev = None
print("\nphase            " + " ".join("%16s" % c[3:] for c in cols[:5]))
for v in rows:
    r = rows[v]
    base = rows[prev] if prev else {c: 0.0 for c in cols}
    print("%-16s " % names[v] + " ".join("%16.1f" % (r.get(c, 0.0) - base.get(c, 0.0)) for c in cols[:5]))
    prev = v
