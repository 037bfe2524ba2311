import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


_CONFIG = None
sys.modules.setdefault("vlog_amd_test_conftest", sys.modules[__name__])   # one handle, however pytest named us


def pytest_configure(config):
    global _CONFIG
    _CONFIG = config
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwhisper_mi355.so)")
    config.addinivalue_line("markers", "slow: long CPU-side test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def terminal_line(msg: str) -> None:
    """One line straight to the terminal, past pytest's output capture (long oracle checks print progress, so a
    runner that watches for silence does not take a minutes-long CPU check for a hang)."""
    if _CONFIG is None:
        return
    capman = _CONFIG.pluginmanager.getplugin("capturemanager")
    if capman is None:
        return
    with capman.global_and_fixture_disabled():
        sys.stderr.write(msg + "\n")
        sys.stderr.flush()
