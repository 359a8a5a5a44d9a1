"""The reference's client integration tests as known answers: the Java
linked-transfer test (IntegrationTest.java:699-781, balances 100 / 49) and the Node client flow
(test.ts:68-341: exists, two-phase post and void, a linked pair repeating an id), transcribed as
data by tests/golden/make_client_fixtures.py.  The oracle must reproduce them (CPU), and so must the
engine through the C ABI (GPU)."""
import pytest

from tests.harness import known_answers
from tests.harness.oracle import OracleEngine

SCENARIOS = known_answers.load()
IDS = [s["name"] for s in SCENARIOS]


def test_fixture_is_what_the_script_writes():
    import json
    import runpy

    path = known_answers.PATH
    committed = open(path).read()
    script = path.replace("client_known_answers.json", "make_client_fixtures.py")
    ns = runpy.run_path(script)
    regenerated = json.dumps({"generated_by": "tests/golden/make_client_fixtures.py",
                              "scenarios": [ns["java"], ns["node"]]}, indent=1) + "\n"
    assert committed == regenerated


@pytest.mark.parametrize("scenario", SCENARIOS, ids=IDS)
def test_oracle_reproduces_client_answers(scenario):
    oracle = OracleEngine()
    try:
        known_answers.run(scenario, oracle)
    finally:
        oracle.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scenario", SCENARIOS, ids=IDS)
def test_gpu_reproduces_client_answers(scenario, gpu_engine_factory):
    known_answers.run(scenario, gpu_engine_factory())
