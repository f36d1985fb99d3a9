import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture
def host_devices():
    """Switch the process to N host (CPU) devices for one test."""
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.runtime.devices import reset_backend

    saved = {k: os.environ.get(k) for k in ("LJS_PLATFORM", "LJS_NUM_DEVICES")}

    def make(n):
        os.environ["LJS_PLATFORM"] = "cpu"
        os.environ["LJS_NUM_DEVICES"] = str(n)
        reset_backend()
        return ljs.devices()

    yield make
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    reset_backend()


@pytest.fixture
def gpu_devices():
    """Switch the process to N (virtual) GPU devices on the local MI355X."""
    import torch
    import learning_jax_sharding_amd as ljs
    from learning_jax_sharding_amd.runtime.devices import reset_backend

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    saved = {k: os.environ.get(k) for k in ("LJS_PLATFORM", "LJS_NUM_DEVICES")}

    def make(n):
        os.environ["LJS_PLATFORM"] = "gpu"
        os.environ["LJS_NUM_DEVICES"] = str(n)
        reset_backend()
        return ljs.devices()

    yield make
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    reset_backend()
