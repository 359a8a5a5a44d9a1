"""Summarise rocprofv3 outputs into profiles/pmc_<tag>.json (per-kernel mean duration and HBM
bytes per launch).  FETCH_SIZE and WRITE_SIZE come from separate --pmc passes (they do not fit in
one pass on gfx950).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE counts 64-B requests and reads ½
of the bytes of wide coalesced streams; we report the raw value and a corrected estimate that
doubles it (the validate kernel's event stream is such a stream; its random 16/32-B probes are
not, so the corrected figure is an upper bound).

usage: python tools/pmc_summary.py <kernel_stats.csv> <fetch_counter_collection.csv>
       <write_counter_collection.csv> <out.json>
"""
import collections
import csv
import json
import sys


def short(name):
    """'void tb_resolve<(unsigned char)129>(PassArgs)' -> 'tb_resolve<129>'; the validate kernels'
    HBM instantiation <false> keeps the plain name, the read-through one <true> gets '_src'."""
    base = name.split("(")[0].replace("void ", "").strip()
    if base.endswith("validate<false>"):
        return base[:-len("<false>")]
    if base.endswith("validate<true>"):
        return base[:-len("<true>")] + "_src"
    if "<" in name.split("(PassArgs")[0]:
        arg = name.split("<", 1)[1].split(">", 1)[0].replace("(unsigned char)", "")
        base = base.split("<")[0] + "<" + arg + ">"
    return base


def main(stats_csv, fetch_csv, write_csv, out):
    res = {"kernels": {}}
    for r in csv.DictReader(open(stats_csv)):
        k = short(r["Name"])
        res["kernels"].setdefault(k, {})
        res["kernels"][k].update({"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                  "total_ms": float(r["TotalDurationNs"]) / 1e6})
    for path, key in ((fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == key:
                agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024)
        for k, v in agg.items():
            res["kernels"].setdefault(k, {})[key.lower() + "_bytes_per_launch"] = sum(v) / len(v)
    for k, d in res["kernels"].items():
        if "fetch_size_bytes_per_launch" in d and "write_size_bytes_per_launch" in d:
            d["hbm_bytes_per_launch_raw"] = d["fetch_size_bytes_per_launch"] + d["write_size_bytes_per_launch"]
            d["hbm_bytes_per_launch"] = 2 * d["fetch_size_bytes_per_launch"] + d["write_size_bytes_per_launch"]
    res["note"] = ("hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half of a wide "
                   "coalesced read; upper bound for random small reads); _raw = FETCH_SIZE + WRITE_SIZE")
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(*sys.argv[1:5])
