import functools
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@functools.lru_cache(maxsize=8)
def net_bytes(seed: int = 1, hd: int = 1024, flags: int = 0) -> bytes:
    from fishnet_amd import synthesize_net
    return synthesize_net(seed, hd, flags)


@pytest.fixture(scope="session")
def big_net_bytes():
    return net_bytes(1, 1024, 0)


@pytest.fixture(scope="session")
def oracle_big(big_net_bytes):
    from oracle.oracle import OracleNet
    return OracleNet(big_net_bytes)


@pytest.fixture(scope="session")
def gpu_eval(big_net_bytes):
    from fishnet_amd import Evaluator, Net
    return Evaluator(Net.from_bytes(big_net_bytes), 0)
