"""Build perf/pmc_<round>.json — the rocprofv3 evidence bench.py's roofline reads (`traffic`,
`rocprof_avg_launch_ms`) — from the kernel-trace and PMC runs of tools/gpu/r0N_prof.sh.

Two legs, each from three runs of one command (kernel trace + stats; FETCH_SIZE alone; WRITE_SIZE
alone — they do not fit in one pass on gfx950, MI355X_MICROARCH.md §HBM):
  headline  bench.py's headline leg (pipelined C2 commits from registered host memory, 64-prepare
            chunks of 523,560 transfers; counters from one 100M-transfer step of the same chunks)
  device    tools/gpu/device_pass.py 100000000 (the bench's device-resident leg: the same 100M
            prepares already in HBM, 512-prepare passes: no host copy in flight while the pass
            kernels run)

Per kernel: rocprof calls and mean duration, and the counters summed over every dispatch divided by
the transfers those dispatches committed (FETCH_SIZE / WRITE_SIZE are KB).  `raw` = FETCH + WRITE;
`fetch_x2` doubles FETCH (gfx950 counts half of a wide coalesced read; an upper bound for random
reads).

usage: python tools/perf_pmc.py <out.json> <round> \
         headline <stats.csv> <fetch.csv> <write.csv> <counter_transfers> <launch_transfers> \
         device   <stats.csv> <fetch.csv> <write.csv> <counter_transfers> <launch_transfers>
"""
import collections
import csv
import json
import sys

PASS_KERNELS = ("tb_transfers_validate", "tb_resolve_lean", "tb_resolve<129>", "tb_apply_legs", "tb_flow",
                "tb_pass_clear", "tb_reply_out")


def short(name):
    """'void tb_resolve<(unsigned char)129>(PassArgs)' -> 'tb_resolve<129>'; validate<false> keeps the
    plain name, validate<true> (read-through from host memory) gets '_src'."""
    base = name.split("(")[0].replace("void ", "").strip()
    if base.endswith("validate<false>"):
        return base[:-len("<false>")]
    if base.endswith("validate<true>"):
        return base[:-len("<true>")] + "_src"
    if "<" in name.split("(PassArgs")[0]:
        arg = name.split("<", 1)[1].split(">", 1)[0].replace("(unsigned char)", "")
        base = base.split("<")[0] + "<" + arg + ">"
    return base


def counter_sums(path, counter):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name", counter) == counter:
            agg[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024
    return agg


def stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": round(float(r["AverageNs"]) / 1e6, 5)}
    return out


def leg(stats_csv, fetch_csv, write_csv, counter_transfers, launch_transfers):
    f, w, s = counter_sums(fetch_csv, "FETCH_SIZE"), counter_sums(write_csv, "WRITE_SIZE"), stats(stats_csv)
    n = int(counter_transfers)
    kernels = {}
    for k in PASS_KERNELS:
        if k not in s and k not in f:
            continue
        fb, wb = f.get(k, 0.0) / n, w.get(k, 0.0) / n
        kernels[k] = {"fetch_per_transfer": round(fb, 1), "write_per_transfer": round(wb, 1),
                      "raw_per_transfer": round(fb + wb, 1), "fetch_x2_per_transfer": round(2 * fb + wb, 1)}
        kernels[k].update({"rocprof_" + a: b for a, b in s.get(k, {}).items()})
    return {"counter_transfers": n, "launch_transfers": int(launch_transfers), "kernels": kernels}


def main(argv):
    out, rnd = argv[0], argv[1]
    res = {"round": rnd,
           "source": "tools/gpu/%s_prof.sh (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE) "
                     "summarised by tools/perf_pmc.py" % rnd,
           "note": "bytes per committed transfer; raw = FETCH_SIZE + WRITE_SIZE; fetch_x2 doubles FETCH_SIZE "
                   "(gfx950 FETCH_SIZE counts half of a wide coalesced read)",
           "legs": {}}
    i = 2
    while i < len(argv):
        name = argv[i]
        res["legs"][name] = leg(*argv[i + 1:i + 6])
        i += 6
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
