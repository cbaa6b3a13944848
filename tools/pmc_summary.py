"""Average each PMC counter per dispatch of the evam_pp kernel over the passes written by tools/pmc.sh."""
import csv
import glob
import json
import os
import sys


def main(d):
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
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
