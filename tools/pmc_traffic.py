"""Per-launch HBM traffic of the bench kernels from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --model M --batch B --precisions fp32,bf16 \
        -o profiles/pmc_traffic_M.json
    (bench.py reads profiles/pmc_traffic_<model>.json and uses it only when the recorded command —
    model, per-GPU batch, world size, precisions, options — matches the running one)

FETCH_SIZE / WRITE_SIZE come from two separate `rocprofv3 --kernel-trace --pmc ...` runs of the same
bench command.  Corrections per MI355X_MICROARCH.md (HBM section, gfx950): FETCH_SIZE (KiB) x 2
(wide 128-B streaming reads are tallied at 64 B), WRITE_SIZE as reported.  Kernels are grouped
under the names bench.py / srk_prof use ("gemm_f32" = every gemm_f32_kernel instantiation, ...);
the value is total bytes / launches, i.e. the same per-launch average as the bench's 'achieved'.
"""
import argparse
import glob
import json
import os
import re
import sqlite3

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_stamp():
    """srk_source_stamp() of the in-tree libsrk.so (the build the counters were collected on); bench.py
    attaches counter data only to a run of the library with the same stamp."""
    import ctypes
    L = ctypes.CDLL(os.path.join(REPO, "speechrecognitionproject_amd", "libsrk.so"))
    L.srk_source_stamp.restype = ctypes.c_char_p
    return L.srk_source_stamp().decode()

GROUPS = {  # srk_prof name -> substrings of the rocprof kernel symbols it covers (GEMMs: _gemm_group)
    "gemm_f32": (), "gemm_bf16": (), "gemm_f16": (), "splitk_reduce": (),
    "gru_fwd_seq": ("gru_fwd_persistent_kernel", "gru_fwd_persistent_dc_kernel"),
    "gru_bwd_seq": ("gru_bwd_persistent_kernel", "gru_bwd_persistent_dc_kernel"),
    "gru_fwd_seq_lp": ("gru_fwd_persistent_lp_kernel", "gru_fwd_persistent_lp2_kernel"),
    "gru_bwd_seq_lp": ("gru_bwd_persistent_lp_kernel", "gru_bwd_persistent_lp2_kernel"),
    "gru_fwd_step": ("gru_fwd_step_kernel",), "gru_bwd_step": ("gru_bwd_step_kernel",),
    "mfcc": ("mfcc3_kernel", "mfcc2_kernel"), "fbank": ("fbank_kernel",), "spec": ("spec_kernel",),
    "conv_fwd": (), "conv_dgrad": (), "conv_wgrad": (), "conv_fwd_lp": (), "conv_dgrad_lp": (), "conv_wgrad_lp": (),
    "adam": ("adam_kernel",), "noise_mix": ("noise_mix_kernel",),
}


def _conv_group(name):
    """conv_gemm_kernel<MODE, BM, BN, BK, VEC, VECB, LP, S16>: MODE 0/1/2 = fwd/dgrad/wgrad, LP != 0 = 16-bit;
    the LDS-DMA ring kernels conv_ring_kernel<MODE, BN> (fp32) and conv_ring16_kernel<MODE, BN, LP> (16-bit)."""
    modes = ("conv_fwd", "conv_dgrad", "conv_wgrad")
    m = re.search(r"conv_gemm_kernel<(\d+),[^,]*,[^,]*,[^,]*,[^,]*,[^,]*,\s*(\d+)", name)
    if m:
        return modes[int(m.group(1))] + ("_lp" if m.group(2) != "0" else "")
    m = re.search(r"conv_ring(16)?_kernel<(\d+)", name)
    if m:
        return modes[int(m.group(2))] + ("_lp" if m.group(1) else "")
    # the row-staged fbanks_cnn conv2 kernels (conv.hip): fp32 = conv_row32_*, 16-bit = conv_row16_*
    m = re.search(r"conv_row(16|32)_(pool|dgrad|wgrad)_kernel", name)
    if m:
        return {"pool": "conv_fwd", "dgrad": "conv_dgrad", "wgrad": "conv_wgrad"}[m.group(2)] + \
            ("_lp" if m.group(1) == "16" else "")
    return None


def _gemm_group(name):
    """The srk_prof GEMM category of a kernel symbol: the operand precision is a template argument
    (gemm_g16_kernel<TA, TB, F16>, gemm_h16_kernel<.., F16>, gemm_lp_kernel<.., F16, PF>, skinny_*<RND, ..>).
    The split-K slab / row-sum reductions (run inside the GEMM's timed scope) are reported on their own."""
    if "splitk_reduce" in name or "rowsum_reduce" in name:
        return "splitk_reduce"
    if "gemm_f32_kernel" in name or "gemm_p32_kernel" in name:
        return "gemm_f32"
    m = re.search(r"skinny_[nmk]_kernel<(\d)", name)
    if m:
        return ("gemm_f32", "gemm_bf16", "gemm_f16")[int(m.group(1))]
    for k, pos in (("gemm_g16_kernel<", 2), ("gemm_h16_kernel<", 5), ("gemm_lp_kernel<", 6)):
        if k in name:
            args = [x.strip() for x in name.split(k, 1)[1].split(">", 1)[0].split(",")]
            return "gemm_f16" if len(args) > pos and args[pos] in ("true", "1") else "gemm_bf16"
    return None


def collect(d, counter):
    db = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    out = {}
    for name, n, tot in c.execute("select kernel_name, count(*), sum(value) from counters_collection where "
                                  "counter_name = ? group by kernel_name", (counter,)):
        cg = _conv_group(name) or _gemm_group(name)
        for g, subs in GROUPS.items():
            if (g == cg) if cg else any(sub in name for sub in subs):
                a = out.setdefault(g, [0, 0.0])
                a[0] += n
                a[1] += tot
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("-o", required=True)
    ap.add_argument("--source", default="")
    ap.add_argument("--model", required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--precisions", default="fp32", help="comma list: the precisions the command timed")
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--sync-bn", action="store_true")
    ap.add_argument("--conv-fwd-fp32", action="store_true")
    ap.add_argument("--merge", action="store_true",
                    help="add to an existing -o file of the same model / batch / world / options (another precision)")
    a = ap.parse_args()
    f, w = collect(a.fetch, "FETCH_SIZE"), collect(a.write, "WRITE_SIZE")
    # bench.py reports this traffic only for a command with the same model / batch / world / options
    res = {"source": a.source, "source_stamp": lib_stamp(),
           "correction": "FETCH_SIZE KiB x 2 x 1024 + WRITE_SIZE KiB x 1024 (gfx950)",
           "command": {"model": a.model, "batch": a.batch, "world": a.world, "precisions": a.precisions.split(","),
                       "sync_bn": bool(a.sync_bn), "conv_fwd_fp32": bool(a.conv_fwd_fp32)},
           "bytes_per_launch": {}}
    for g in sorted(set(f) & set(w)):
        fb = 2.0 * 1024.0 * f[g][1] / f[g][0]
        wb = 1024.0 * w[g][1] / w[g][0]
        res["bytes_per_launch"][g] = {"fetch": round(fb), "write": round(wb), "total": round(fb + wb),
                                      "launches": f[g][0]}
    if a.merge and os.path.exists(a.o):
        with open(a.o) as fh:
            old = json.load(fh)
        oc, nc = old.get("command", {}), res["command"]
        if (all(oc.get(k) == nc[k] for k in ("model", "batch", "world", "sync_bn", "conv_fwd_fp32"))
                and old.get("source_stamp") == res["source_stamp"]):
            nc["precisions"] = sorted(set(oc.get("precisions", [])) | set(nc["precisions"]))
            res["source"] = "%s + %s" % (old.get("source", ""), a.source)
            res["bytes_per_launch"] = dict(old.get("bytes_per_launch", {}), **res["bytes_per_launch"])
    with open(a.o, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
