"""Multi-rank sharding on the GPU: two ranks (processes) over gloo, both engines on cuda:0 (one
GPU box), exercising the real routing kernels (tb_route_classify / _offsets / _scatter /
_replies), the routed commit and the prefetch / upsert write-back primitives — checked against one
CPU oracle committing the concatenated prepares (tests/harness/shard_runner.py)."""
import pytest

from tests.test_sharded import CLEAN, run_world

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_sharded_clean(tmp_path, seed):
    v = run_world(tmp_path, "gpu", 2, dict(seed=seed, n_accounts=64, n_transfer_batches=8, **CLEAN))
    assert v["ok"], v["problems"]
    assert v["clean"] > 0 and v["dirty"] == 0 and v["split"] == 0


def test_gpu_sharded_clean_large_batches(tmp_path):
    # Full-size prepares: many route workgroups, duplicate ids across ranks and passes.
    v = run_world(tmp_path, "gpu", 2, dict(seed=21, n_accounts=512, n_transfer_batches=8, batch_len=(4000, 8190),
                                           p_dup=0.02, **CLEAN))
    assert v["ok"], v["problems"]
    assert v["clean"] > 0


@pytest.mark.parametrize("seed", [3, 4])
def test_gpu_sharded_mixed(tmp_path, seed):
    v = run_world(tmp_path, "gpu", 2, dict(seed=seed, n_accounts=64, n_transfer_batches=10))
    assert v["ok"], v["problems"]
    assert v["split"] > 0 and v["dirty"] == 0  # dependent subsequences sequenced, no whole-pass gather


def test_gpu_sharded_interleaved(tmp_path):
    v = run_world(tmp_path, "gpu", 2, dict(seed=11, n_accounts=32, n_transfer_batches=14, p_linked=0.02,
                                           p_pending=0.3, p_post_void=0.1, p_balancing=0.0, p_limit=0.0),
                  max_prepares=1)
    assert v["ok"], v["problems"]
    assert v["clean"] > 0 and v["split"] > 0


def test_gpu_sharded_three_ranks(tmp_path):
    v = run_world(tmp_path, "gpu", 3, dict(seed=12, n_accounts=64, n_transfer_batches=9, **CLEAN), max_prepares=3)
    assert v["ok"], v["problems"]


def test_gpu_sharded_dependent_kinds(tmp_path):
    # Split dirty passes with every dependency class and cross-rank duplicate ids (demotion), on the
    # real kernels (tb_route_dependents, the skip-mask route plan, tb_route_homes).
    v = run_world(tmp_path, "gpu", 2, dict(seed=31, n_accounts=24, n_transfer_batches=12, p_linked=0.25, p_limit=0.3,
                                           p_balancing=0.1, p_pending=0.4, p_post_void=0.3, p_dup=0.15, id_space=400))
    assert v["ok"], v["problems"]
    assert v["split"] > 0 and v["demoted"] > 0


def test_gpu_sharded_rccl_one_rank(tmp_path):
    """The protocol over RCCL (backend "nccl"): device tensors for every collective, torch's current
    stream synchronised before each.  One rank (the box has one GPU; RCCL refuses two ranks on one
    device), every pass kind: clean and split passes through the real kernels and collectives."""
    v = run_world(tmp_path, "gpu", 1, dict(seed=41, n_accounts=64, n_transfer_batches=10), dist_backend="nccl")
    assert v["ok"], v["problems"]
    assert v["clean"] + v["split"] + v["dirty"] > 0
