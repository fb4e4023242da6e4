"""tools/ab.sh's parity gate hands a candidate's launch knobs to the GPU suite
through BWRT_AB_ENV; tests/conftest.py strips every other BWRT_* variable
(a stray knob would change which kernel a default-policy test checks) and
re-applies those, before the first test and after every test.  The library
reads its knobs with getenv in rt_create, in the test process, so a knob in
that process's environment is a knob the gate's renders use."""
import json
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _expect():
    return json.loads(os.environ.get("AB_PROBE_EXPECT", "null"))


@pytest.mark.skipif(_expect() is None, reason="probe: run by test_ab_knobs_reach_the_tests")
@pytest.mark.parametrize("i", [0, 1])  # the second run follows the per-test reset
def test_probe(i):
    want = _expect()
    got = {k: v for k, v in os.environ.items() if k.startswith("BWRT_") and k not in ("BWRT_LIB", "BWRT_TUNING",
                                                                                        "BWRT_AB_ENV")}
    assert got == want
    os.environ["BWRT_LEFT_BEHIND"] = "1"  # the autouse fixture must drop it


def test_ab_knobs_reach_the_tests():
    env = dict(os.environ)
    env.update(BWRT_AB_ENV="BWRT_REFILL=32,BWRT_GREC=1", BWRT_BLOCK="128",
               AB_PROBE_EXPECT=json.dumps({"BWRT_REFILL": "32", "BWRT_GREC": "1"}))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(REPO, "tests", "test_ab_env.py"), "-k", "probe"],
                       env=env, cwd=REPO, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "2 passed" in r.stdout


def test_ab_sh_passes_knobs_through_ab_env():
    """ab.sh's SUBSET gate names the knobs in BWRT_AB_ENV (not as bare
    variables, which conftest would strip)."""
    text = open(os.path.join(REPO, "tools", "ab.sh")).read()
    gate = [ln for ln in text.splitlines() if "pytest" in ln and "env " in ln]
    assert gate and all('BWRT_AB_ENV="$envs"' in ln for ln in gate)
    # the spec's third field (comma list of K=V) is what lands in BWRT_AB_ENV
    spec = "cand:base:BWRT_REFILL=32,BWRT_GREC=1"
    out = subprocess.run(["bash", "-c", 'IFS=: read -r label var envs <<< "$1"; printf %s "$envs"', "_", spec],
                         capture_output=True, text=True, check=True).stdout
    from conftest import ab_knobs
    assert ab_knobs(out) == {"BWRT_REFILL": "32", "BWRT_GREC": "1"}
    with pytest.raises(ValueError):
        ab_knobs("NOT_A_KNOB=1")
    assert re.search(r"BWRT_AB_ENV", open(os.path.join(REPO, "tests", "conftest.py")).read())
