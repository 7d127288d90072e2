"""bench.py's choice of the timed interval (CPU only: no launch).

The bench reports the HIP event interval on the decoder's stream (max over ranks); an interval longer
than the host wall clock around the same launches cannot be right, and the wall clock is reported then
(profiles/r06/rehearsal_g2/ holds the two-ranks-on-one-GPU runs that motivated the check).
"""
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # module level: imports and constants only
    return mod


def test_events_kept_when_inside_the_wall_clock(bench):
    assert bench.step_time(0.0017, 0.0020) == (0.0017, "hip events")
    assert bench.step_time(0.0020, 0.0020)[1] == "hip events"
    assert bench.step_time(0.00201, 0.0020)[1] == "hip events"  # within the 2 % slack


def test_wall_clock_when_events_exceed_it(bench):
    t, timer = bench.step_time(100.0, 2.0)
    assert t == 2.0 and timer.startswith("host wall clock")
