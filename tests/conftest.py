import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "miotts-llama.cpp_amd")
for p in (os.path.join(PKG, "python"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def device():
    import miotts_amd as m
    if m.device_count() < 1:
        pytest.fail("gpu test run without a visible HIP device")
    d = m.Device(0)
    yield d
    d.close()


@pytest.fixture(scope="session")
def synth_llm_path(tmp_path_factory):
    """synth_llm_path(preset) -> path of the synthetic LLM GGUF of that preset (seed 1),
    written once per test session (the 1.7B / 2.6B files take seconds to synthesize)."""
    import miotts_amd as m
    d = tmp_path_factory.mktemp("llm_models")
    cache = {}

    def get(preset: int) -> str:
        if preset not in cache:
            cache[preset] = m.synth_llm(str(d / f"llm{preset}.gguf"), preset, 1)
        return cache[preset]

    return get
