"""bench.py's multi-GPU launch on the CPU (no GPU call): `--gpus N` with the per-process engine
starts N ranks itself, and under torchrun every rank joins the process group (the driver's scaling
run launches `torch.distributed.run ... bench.py --gpus N`)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(cmd):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    return lines[0]


def test_gpus_n_self_launches_ranks():
    v = _run([sys.executable, BENCH, "--gpus", "2", "--engine", "ranks", "--dist-backend", "gloo", "--same-device",
              "--launch-check"])
    assert v["world"] == 2 and v["ranks"] == [0, 1] and v["worlds"] == [2]


def test_torchrun_launch_matches_gpus():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    v = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "3",
              "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "3", "--launch-check"])
    assert v["world"] == 3 and v["ranks"] == [0, 1, 2] and v["engine"] == "node"
