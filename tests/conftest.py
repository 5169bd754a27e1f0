"""Test configuration.

Markers: ``gpu`` -- needs an MI355X (run by the driver with ``-m gpu`` on a GPU box);
everything else runs on CPU (multi-process tests use the shared-memory host
transport of the ``mi355x`` backend, world sizes 1/2/4/8, spawn + 127.0.0.1
rendezvous -- the reference's own fixture pattern, main.py:90-108).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD Instinct MI355X GPU")
    config.addinivalue_line("markers", "slow: long-running test")
