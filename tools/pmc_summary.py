"""Average each PMC counter per dispatch of the evam_pp kernel over the passes written by tools/pmc.sh."""
import csv
import glob
import json
import os
import sys


def main(d, config=None, frames_per_launch=None, traffic_json=None, pool_sets=1):
    vals = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if "evam_pp" not in r.get("Kernel_Name", ""):
                continue
            name = r["Counter_Name"]
            vals.setdefault(name, {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[name][r["Dispatch_Id"]] += float(r["Counter_Value"])
    out = {k: sum(v.values()) / len(v) for k, v in vals.items() if v}
    for k in sorted(out):
        print(f"{k:28s} {out[k]:.6g}")
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        fetch = out["FETCH_SIZE"] * 1024 * 2  # KB; x2: gfx950 FETCH_SIZE reads half of wide streaming reads
        write = out["WRITE_SIZE"] * 1024
        print(f"hbm_bytes_per_launch (fetch x2 corrected + write) = {fetch + write:.6g}  (fetch {fetch:.6g}, write {write:.6g})")
        if traffic_json and config:
            t = json.load(open(traffic_json)) if os.path.exists(traffic_json) else {}
            t[config] = {"frames_per_launch": frames_per_launch, "pool_sets": pool_sets,
                         "hbm_bytes_per_launch": int(fetch + write),
                         "fetch_bytes": int(fetch), "write_bytes": int(write),
                         "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, mean per dispatch "
                                   "of the evam_pp kernel; FETCH_SIZE (KB) x2 for the gfx950 half-count of wide "
                                   "streaming reads (MI355X_MICROARCH.md, HBM), WRITE_SIZE (KB) as is",
                         "source": os.path.relpath(d)}
            json.dump(t, open(traffic_json, "w"), indent=1)
    if "SQ_INSTS_VALU" in out and traffic_json and config:
        vj = os.path.join(os.path.dirname(traffic_json), "pmc_valu.json")
        t = json.load(open(vj)) if os.path.exists(vj) else {}
        t[config] = {"frames_per_launch": frames_per_launch, "pool_sets": pool_sets,
                     "valu_insts_per_launch": int(out["SQ_INSTS_VALU"]),
                     **{k: out[k] for k in ("SQ_ACTIVE_INST_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "GRBM_GUI_ACTIVE",
                                            "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES") if k in out},
                     "method": "rocprofv3 --pmc SQ_INSTS_VALU ..., mean per dispatch of the evam_pp kernel "
                               "(wave-level VALU instructions)",
                     "source": os.path.relpath(d)}
        json.dump(t, open(vj, "w"), indent=1)
        print(f"valu_insts_per_launch = {int(out['SQ_INSTS_VALU'])}")
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], *(a[1:2] or [None]), *([int(a[2])] if len(a) > 2 else [None]), *(a[3:4] or [None]),
         *([int(a[4])] if len(a) > 4 else []))
