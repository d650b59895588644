import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libkcc.so")


def have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def init_torch_first():
    """Initialise torch's HIP runtime (bundled with the wheel) before libkcc's (/opt/rocm):
    torch's fails to come up in a process where the other one initialised first."""
    import torch
    torch.cuda.init()


@pytest.fixture(scope="session")
def engine():
    """One libkcc context for the whole GPU session (device 0)."""
    init_torch_first()
    from kubernetesclustercapacity_amd import CapacityEngine
    eng = CapacityEngine(0, 1)
    yield eng
    eng.close()
