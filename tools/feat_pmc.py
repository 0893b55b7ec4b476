"""Feature-kernel (K1-K3) PMC summary for bench.py's feature_roofline -> profiles/pmc_feature.json.

    python tools/feat_pmc.py DIR -o profiles/pmc_feature.json --clips 65536

DIR holds one rocprofv3 `--kernel-trace --pmc` pass per sub-directory, named p<pass>_<feature>
(tools/feat_pmc.sh: FETCH_SIZE alone, WRITE_SIZE alone, then two SQ groups), each a run of
`python3 tools/mfcc_only.py <feature> <clips>` (the models' layouts, as bench.py times them).

Per feature kernel: HBM bytes per launch and per clip, and the SQ counters per clip
(SQ_INSTS_VALU, SQ_WAIT_INST_ANY, ...; counters summed over the dispatch's SEs / XCDs, then averaged
over dispatches).  FETCH_SIZE correction (MI355X_MICROARCH.md, HBM section): gfx950 tallies a wide
16-B/lane streaming read at half its bytes.  The feature kernels read the clips with 8-B/lane loads,
so instead of assuming a factor the script calibrates it on the one quantity it knows exactly: the
PCM input (64,000 B/clip, 4.2 GB per launch — far past the 256 MB MALL, so read from HBM at least
once).  A raw FETCH_SIZE below 0.75x the input bytes is doubled; the raw value is kept alongside.
"""
import argparse
import glob
import json
import os
import sqlite3

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_stamp():
    """srk_source_stamp() of the in-tree libsrk.so (the build the counters were collected on); bench.py
    attaches counter data only to a run of the library with the same stamp."""
    import ctypes
    L = ctypes.CDLL(os.path.join(REPO, "speechrecognitionproject_amd", "libsrk.so"))
    L.srk_source_stamp.restype = ctypes.c_char_p
    return L.srk_source_stamp().decode()

KERNELS = {"mfcc": ("mfcc3_kernel", "mfcc4_kernel", "mfcc2_kernel"), "fbank": ("fbank_kernel",),
           "spec": ("spec_kernel",)}
PCM_BYTES_PER_CLIP = 64000


def per_dispatch(d, feature):
    """{counter: mean value per dispatch of the feature kernel}, mean duration (ns), dispatches."""
    acc, dur = {}, {}
    for db in sorted(glob.glob(os.path.join(d, "p*_" + feature, "**", "*.db"), recursive=True)):
        con = sqlite3.connect(db)
        for kname, counter, value, ev, ns in con.execute(
                "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
            if not any(k in kname for k in KERNELS[feature]):
                continue
            key = (db, ev)
            acc.setdefault(counter, {})
            acc[counter][key] = acc[counter].get(key, 0.0) + float(value)
            dur[key] = float(ns)
    means = {c: sum(v.values()) / len(v) for c, v in acc.items()}
    return means, (sum(dur.values()) / len(dur) if dur else None), len(dur)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", required=True)
    ap.add_argument("--clips", type=int, required=True)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    res = {"source": a.source, "source_stamp": lib_stamp(),
           "command": "python3 tools/mfcc_only.py <feature> %d" % a.clips,
           "clips_per_launch": a.clips, "kernels": {}}
    for feature in KERNELS:
        m, ns, nd = per_dispatch(a.dir, feature)
        if not m:
            continue
        n = float(a.clips)
        ent = {"dispatches": nd, "mean_duration_us_under_pmc": round(ns / 1e3, 1) if ns else None}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            raw = 1024.0 * m["FETCH_SIZE"]
            factor = 2.0 if raw < 0.75 * PCM_BYTES_PER_CLIP * n else 1.0
            fetch, write = factor * raw, 1024.0 * m["WRITE_SIZE"]
            ent.update({"fetch_bytes_raw": round(raw), "fetch_factor": factor, "fetch_bytes": round(fetch),
                        "write_bytes": round(write), "traffic_per_launch": round(fetch + write),
                        "traffic_per_clip": round((fetch + write) / n, 1)})
        per_clip = {c: round(v / n, 1) for c, v in sorted(m.items()) if c.startswith("SQ_")}
        if per_clip:
            ent["per_clip"] = per_clip
            if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_INST_ANY" in m:
                ent["wait_inst_any_frac_of_wave_cycles"] = round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
            if "SQ_WAVE_CYCLES" in m and "SQ_ACTIVE_INST_ANY" in m:
                ent["active_inst_any_frac_of_wave_cycles"] = round(m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)
        res["kernels"][feature] = ent
    with open(a.o, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
