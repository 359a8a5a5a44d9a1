"""Per-transfer HBM bytes of the pass kernels in device-resident C2 passes (tools/gpu/device_pass.py
under `profile.sh dfetch|dwrite`): the counters summed over every dispatch of a kernel, divided by
the transfers those dispatches committed (FETCH_SIZE and WRITE_SIZE are in KB).

usage: python tools/gpu/device_pmc.py <fetch.csv> <write.csv> <transfers> <out.json>
"""
import collections
import csv
import json
import sys

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), ".."))
from pmc_summary import short  # noqa: E402

PASS_KERNELS = ("tb_transfers_validate", "tb_resolve<129>", "tb_apply_legs", "tb_flow", "tb_pass_clear")


def sums(path):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024
    return agg


def main(fetch_csv, write_csv, transfers, out):
    f, w = sums(fetch_csv), sums(write_csv)
    transfers = int(transfers)
    res = {"source": "tools/gpu/profile.sh dfetch|dwrite: tools/gpu/device_pass.py, C2, 1M accounts, %d transfers "
                     "already in HBM, 512-prepare passes, tables sized for 100M transfers" % transfers,
           "note": "bytes per committed transfer; raw = FETCH_SIZE + WRITE_SIZE, fetch_x2 doubles FETCH_SIZE "
                   "(gfx950 FETCH_SIZE counts half of a wide coalesced read; an upper bound for random reads)",
           "kernels": {}}
    for k in PASS_KERNELS:
        fb, wb = f.get(k, 0.0) / transfers, w.get(k, 0.0) / transfers
        res["kernels"][k] = {"fetch_per_transfer": round(fb, 1), "write_per_transfer": round(wb, 1),
                             "raw_per_transfer": round(fb + wb, 1), "fetch_x2_per_transfer": round(2 * fb + wb, 1)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(k, v)


if __name__ == "__main__":
    main(*sys.argv[1:5])
