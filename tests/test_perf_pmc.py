"""The roofline's `traffic` evidence (VERDICT r3 What's weak #3): the round's perf/pmc_rNN.json
(bench.py's PMC_FILE) travels with the tree and holds every pass kernel the bench's rooflines name,
bench.py reads it (and says so loudly when an entry is missing), and tools/perf_pmc.py builds it
from rocprofv3's CSVs."""
import csv
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _pmc_file():
    sys.argv = ["bench.py"]
    return _load("bench_for_pmc_file", "bench.py").PMC_FILE


def test_committed_pmc_file_covers_the_rooflines():
    name = _pmc_file()
    d = json.load(open(os.path.join(ROOT, name)))
    for leg in ("headline", "device"):
        kernels = d["legs"][leg]["kernels"]
        for k in ("tb_transfers_validate", "tb_resolve<129>", "tb_apply_legs"):
            e = kernels[k]
            assert e["rocprof_calls"] > 0 and e["rocprof_avg_ms"] > 0
            assert e["fetch_x2_per_transfer"] >= e["raw_per_transfer"]
        # the resolve stage's bytes: tb_resolve_lean's on a clean legs pass (round 6: tb_resolve<129>
        # then only exits early), tb_resolve<129>'s otherwise
        for k in ("tb_transfers_validate", "tb_apply_legs"):
            assert kernels[k]["raw_per_transfer"] > 0
        lean = kernels.get("tb_resolve_lean", {})
        assert max(lean.get("raw_per_transfer", 0), kernels["tb_resolve<129>"]["raw_per_transfer"]) > 0
    # the gitignore / gpurunignore must let it travel to the GPU box
    ignore = open(os.path.join(ROOT, ".gpurunignore")).read().split()
    assert not any(p.strip("./") in ("perf", "perf/", name) for p in ignore)


def test_bench_reads_the_file_and_fails_loudly(capsys, monkeypatch):
    sys.argv = ["bench.py"]
    bench = _load("bench_under_test", "bench.py")
    out = bench.load_pmc("headline", "tb_transfers_validate", 523560)
    assert out["traffic"] > 0 and out["rocprof_avg_launch_ms"] > 0 and "traffic_error" not in out
    missing = bench.load_pmc("headline", "no_such_kernel", 523560)
    assert missing["traffic"] is None and os.path.basename(bench.PMC_FILE) in missing["traffic_error"]
    assert "no PMC traffic" in capsys.readouterr().err
    monkeypatch.setattr(bench, "PMC_FILE", os.path.join("perf", "absent.json"))
    assert bench.load_pmc("device", "tb_transfers_validate", 1)["traffic"] is None


def test_perf_pmc_summarises_rocprof_csvs(tmp_path):
    pmc = _load("perf_pmc_under_test", os.path.join("tools", "perf_pmc.py"))
    stats = tmp_path / "stats.csv"
    with open(stats, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "AverageNs"])
        w.writerow(["void tb_transfers_validate<false>(PassArgs)", 2, 90000])
        w.writerow(["void tb_resolve<(unsigned char)129>(PassArgs)", 2, 40000])
    for name, counter, kb in (("fetch.csv", "FETCH_SIZE", 100.0), ("write.csv", "WRITE_SIZE", 50.0)):
        with open(tmp_path / name, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value"])
            for _ in range(2):
                w.writerow(["void tb_transfers_validate<false>(PassArgs)", counter, kb])
    out = tmp_path / "pmc.json"
    pmc.main([str(out), "rX", "headline", str(stats), str(tmp_path / "fetch.csv"), str(tmp_path / "write.csv"),
              "1024", "512"])
    d = json.load(open(out))
    v = d["legs"]["headline"]["kernels"]["tb_transfers_validate"]
    assert v["fetch_per_transfer"] == 200.0 and v["write_per_transfer"] == 100.0  # 2 x KB x 1024 / 1024
    assert v["raw_per_transfer"] == 300.0 and v["fetch_x2_per_transfer"] == 500.0
    assert v["rocprof_calls"] == 2 and v["rocprof_avg_ms"] == 0.09
    assert d["legs"]["headline"]["kernels"]["tb_resolve<129>"]["rocprof_avg_ms"] == 0.04
