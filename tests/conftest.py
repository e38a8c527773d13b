import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if os.path.join(ROOT, "tests") not in sys.path:
    sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    """The C oracle (test infrastructure), built on demand with gcc."""
    from antidote_amd import _abi
    so = os.path.join(ROOT, "oracle", "liboracle.so")
    src = os.path.join(ROOT, "oracle", "oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return _abi.bind(ctypes.CDLL(so), _abi.ORACLE_PROTOTYPES)


@pytest.fixture(scope="session")
def eng():
    """One engine context on cuda:0 for every GPU test of the session."""
    from antidote_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture
def monkeypatch(monkeypatch):
    """pytest's monkeypatch, with every environment change passed on to the
    library's cached AGN_* knobs (agn_env_reload)."""
    from antidote_amd import _lib
    setenv, delenv = monkeypatch.setenv, monkeypatch.delenv

    def _setenv(*a, **k):
        setenv(*a, **k)
        _lib.env_changed()

    def _delenv(*a, **k):
        delenv(*a, **k)
        _lib.env_changed()
    monkeypatch.setenv, monkeypatch.delenv = _setenv, _delenv
    yield monkeypatch


@pytest.fixture(autouse=True)
def _knobs_current():
    """The previous test's monkeypatch undo has restored the environment:
    the library re-reads its knobs before this test runs."""
    from antidote_amd import _lib
    _lib.env_changed()
    yield
