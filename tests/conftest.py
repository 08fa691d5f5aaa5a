import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP pass library)")


@pytest.fixture(scope="session")
def soc():
    import soc_real_time_renderer_amd as m
    m.lib()
    return m


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    return o


@pytest.fixture(autouse=True)
def _tuning_knobs_fresh(monkeypatch):
    """Tests that set SOC_* tuning knobs (monkeypatch.setenv, then soc.reload_tuning()) leave no cached value
    behind: the knob cache is dropped after the environment is restored."""
    yield
    monkeypatch.undo()
    if "soc_real_time_renderer_amd" in sys.modules:
        m = sys.modules["soc_real_time_renderer_amd"]
        if getattr(m, "_LIB", None) is not None:
            m.reload_tuning()


def pytest_terminal_summary(terminalreporter):
    """The achieved errors of the full-frame parity checks (helpers.frame_parity), one JSON line per frame."""
    import json
    h = sys.modules.get("helpers")
    reps = getattr(h, "PARITY_REPORTS", None) if h else None
    if reps:
        terminalreporter.section("full-frame parity: achieved errors")
        for r in reps:
            terminalreporter.write_line(json.dumps(r))
