"""CPU: every seeded differential workload of tests/test_gpu_differential.py is well-formed and the
oracle commits it (so a generator bug shows up here, not first on the GPU box)."""
import pytest

from tests.harness.oracle import OracleEngine, OraclePanic
from tests.harness.workload import make_scenario, run_oracle
from tests.test_gpu_differential import CONFIGS


@pytest.mark.parametrize("config", sorted(CONFIGS))
def test_oracle_commits_differential_workloads(config):
    for seed in (1, 2, 3):
        sc = make_scenario(seed * 7919 + sum(map(ord, config)), **CONFIGS[config])
        try:
            replies = run_oracle(sc, OracleEngine())
        except OraclePanic:
            continue  # the GPU test then expects EnginePanic
        assert len(replies) == sum(1 for s in sc.steps if s[0] == "commit")
